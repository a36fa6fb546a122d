#!/bin/bash
# (dev tool, runs here, not on the GPU box) usage: tools/gpurun_wait.sh OUTFILE [gpurun args] -- CMD
# gpurun with a wait-and-retry only when no command ran (no slot / box not prepared / backoff)
OUT=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > "$OUT" 2>&1
  if grep -q "nothing was charged\|stopped responding while being prepared\|backing off\|was taken away by the GPU service\|has no free box right now" "$OUT"; then
    sleep 90; continue
  fi
  break
done
tail -12 "$OUT"
