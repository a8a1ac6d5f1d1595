#!/bin/bash
# summary of gpurun_out/pytest_gpu.log + bench.log
tail -2 gpurun_out/pytest_gpu.log
tail -1 gpurun_out/bench.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; e=d.get('extras')
print('value %.4g frac %.3f launch %.1fus'%(d['value'], r['frac'], r['avg_launch_us']))
if e: print('unfused %.3g'%e['unfused_graph']['value'], 'large step frac %.3f'%e['large_batch']['step_kernel']['frac'], 'large rollout %.3g frac %.3f'%(e['large_batch']['rollout_kernel']['env_steps_per_s'], e['large_batch']['rollout_kernel']['frac']))"
