#!/bin/bash
# gpurun with retries on transient infra failures (status transient / rc 3). Usage: gpr.sh OUTFILE TIMEOUT CMD
out=$1; to=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|no box or slot" $out && ! grep -q "status=ok" $out; then
    echo "[retry $i] $(grep -o 'status=[a-z]*' $out | tail -1) $(tail -2 $out | head -1)" >> $out.retries
    sleep $((30 * i)); continue
  fi
  break
done
exit $rc
