mkdir -p gpurun_out/sweep2
for P in 25 50 150 300 600 850; do
  timeout -k 10 200 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline --pull-permille $P > gpurun_out/sweep2/p${P}.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sweep2/p${P}.json'));print('pull_permille=$P', d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
done
