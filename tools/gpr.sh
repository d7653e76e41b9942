#!/bin/bash
# gpurun, re-submitted only while the pool reports no free box or slot (status transient / rc 3: nothing ran,
# nothing was charged).  A call that ran -- whatever its exit status -- is never repeated.
# Usage: gpr.sh OUTFILE TIMEOUT CMD
out=$1; to=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|no box or slot\|GPU slot(s) on this pod are busy\|backing off" $out && ! grep -q "status=ok" $out; then
    echo "[retry $i] $(date +%H:%M:%S) $(grep -o 'status=[a-z]*' $out | tail -1) $(tail -2 $out | head -1 | cut -c1-120)" >> $out.retries
    sleep 75; continue
  fi
  break
done
exit $rc
