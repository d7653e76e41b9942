mkdir -p gpurun_out/sweep
for U in 1 2 4; do
  for F in 1 400 1000; do
    GOSSIP_PULL_UNROLL=$U timeout -k 10 200 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline --front-permille $F > gpurun_out/sweep/u${U}_f${F}.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/sweep/u${U}_f${F}.json'));print('U=$U F=$F', d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
  done
done
