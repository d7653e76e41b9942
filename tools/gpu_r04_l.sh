#!/bin/bash
# Round 4: bench lines of configs 4 and 5 after the row-dealt dense rounds; A/B of the apply's bin size.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04l}; mkdir -p $O
for c in 4 5; do
  timeout -k 10 400 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -20 $O/bench_c$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_c$c.json').read().splitlines()[-1]);r=d['roofline'];print($c, d['value'], 'GTEPS', d['ms_per_step'], 'ms', 'frac', r.get('frac'), 'step', r.get('step_frac'), r.get('kernel_ms_per_step'))"
done
for bw in 9216 12288; do
  timeout -k 10 300 python3 -u tools/round_profile.py 4 t.bin_words=$bw > $O/rounds_c4_bw$bw.txt 2>&1 || { tail -20 $O/rounds_c4_bw$bw.txt; exit 1; }
  echo "== bin_words $bw"; grep -E "^(5|6) " $O/rounds_c4_bw$bw.txt | cut -c1-200
done
