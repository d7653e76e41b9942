#!/bin/bash
# usage: sweep_env.sh "<ENV1>" "<ENV2>" ...   (each arg: space-separated VAR=VAL list, "-" = none)
# Runs the default bench (no cpu baseline) once per setting; prints ms/step and per-kernel ms.
set -o pipefail
mkdir -p gpurun_out/sweep
i=0
for setting in "$@"; do
  i=$((i+1))
  [ "$setting" = "-" ] && setting=""
  env $setting timeout -k 10 200 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/sweep/s$i.json 2> gpurun_out/sweep/s$i.err || { tail -5 gpurun_out/sweep/s$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/sweep/s$i.json'));print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])" "[$setting]"
done
