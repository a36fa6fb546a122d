#!/bin/bash
# (dev tool, runs here, not on the GPU box) usage: tools/gpurun_wait2.sh OUTFILE [gpurun args] -- CMD
# gpurun, waiting and trying again only when no command ran (no free slot or box, a box lost
# while being prepared, the service's back-off); waits as long as the message asks
OUT=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" > "$OUT" 2>&1
  if grep -q "nothing was charged\|stopped responding while being prepared\|backing off\|was taken away by the GPU service\|has no free box right now" "$OUT"; then
    w=$(grep -o "retry in [0-9]*s" "$OUT" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-80} + 15 ))
    continue
  fi
  break
done
tail -12 "$OUT"
