#!/bin/bash
# Round evidence for profiles/<tag>/: kernel-trace stats of the default bench,
# FETCH_SIZE and WRITE_SIZE in separate passes, calibration passes, summary.
# usage: bash tools/gpu_profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/calib_fetch tools/calib_fetch.hip 2>/dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4_trace -o run -- python3 -u bench.py --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/bench_trace.err || { tail -5 $OUT/bench_trace.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c4_fetch -o run -- python3 -u bench.py --no-cpu-baseline --no-timing > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err || { tail -5 $OUT/bench_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c4_write -o run -- python3 -u bench.py --no-cpu-baseline --no-timing > $OUT/bench_write.json 2> $OUT/bench_write.err || { tail -5 $OUT/bench_write.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o run -- /tmp/calib_fetch > $OUT/calib_fetch_timing.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o run -- /tmp/calib_fetch > /dev/null 2>&1 || exit 1
python3 tools/pmc_summary.py $OUT $OUT/config4_pmc_summary.json c4 || exit 1
cat $OUT/bench_trace.json
echo profile-done
