mkdir -p gpurun_out/sweep3
for H in 32 64 128 256; do
  for c in 2 3 4; do
    GOSSIP_HEAVY_DEGREE=$H timeout -k 10 200 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep3/h${H}_c${c}.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/sweep3/h${H}_c${c}.json'));print('heavy=$H config=$c', d['ms_per_step'], {k: v for k, v in d['roofline']['kernel_ms_per_step'].items() if v > 0.05})"
  done
done
