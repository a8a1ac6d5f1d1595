import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from golden_util import Fixture
from optimax_rogue_amd import EnvConfig
from optimax_rogue_amd.engine import BatchedEngine
fx = Fixture("c1_random_32")
e = BatchedEngine(EnvConfig.from_dict(fx.cfg), fx.G, seed=fx.seed, game_offset=fx.game_offset, device=torch.device("cuda", 0))
T = fx.T
act = torch.zeros((T, fx.G, 2), dtype=torch.int8, device=e.device)
e.rollout(T, *fx.policy, act=act)
a = act.cpu().numpy()
print("G", fx.G, "policy", fx.policy)
shown = 0
for t in range(T):
    bad = np.nonzero((a[t] != fx.actions[t]).any(1))[0]
    if len(bad) == 0: continue
    shown += 1
    if shown > 8: break
    print(t, len(bad), bad[:8], a[t][bad[:4]].tolist(), fx.actions[t][bad[:4]].tolist())
print("T", T, "status at end", e.status.cpu().numpy(), "tick", e.tick.cpu().numpy(), "ep", e.episode.cpu().numpy())
print("fixture tick/status around first bad:", [ (int(fx.state(t)["tick"][0]), int(fx.state(t)["status"][0])) for t in range(995, 1005)])
