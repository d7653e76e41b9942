#!/bin/bash
# gpurun, re-submitted only while the pool reports no free box or slot, or backs off (status transient: nothing
# ran, nothing was charged).  A call that ran -- whatever its exit status -- is never repeated.
# Usage: gpr.sh OUTFILE TIMEOUT CMD
out=$1; to=$2; shift 2
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|no box or slot\|GPU slot(s) on this pod are busy\|backing off" $out && ! grep -q "status=ok" $out; then
    wait_s=$(grep -o "retry in [0-9]*s" $out | tail -1 | grep -o "[0-9]*")
    echo "[retry $i] $(date +%H:%M:%S) $(grep -o 'status=[a-z]*' $out | tail -1) wait ${wait_s:-75}s $(tail -2 $out | head -1 | cut -c1-100)" >> $out.retries
    sleep $(( ${wait_s:-65} + 10 )); continue
  fi
  break
done
exit $rc
