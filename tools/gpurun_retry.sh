#!/bin/bash
# Runs one gpurun call, retrying ONLY when no box or slot was free (gpurun
# reports status=transient and "nothing was charged" / "retry": nothing ran).
# A call that ran -- whatever its outcome -- is never repeated.
#   tools/gpurun_retry.sh <out-file> <timeout-s> '<command>'
OUT=${1:?out}; TMO=${2:?timeout}; CMD=${3:?command}
for attempt in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if grep -q "status=transient" "$OUT" && grep -qE "nothing was charged|retry" "$OUT" \
      && ! grep -q "run [1-9]" "$OUT"; then
    echo "attempt $attempt: no box/slot (rc=$rc), waiting" >> "$OUT.retries"
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
