#!/bin/bash
# The one GPU driver (round 6; it replaces the per-call scripts of rounds 3-5, which stay in the history).
# Runs on the GPU box from the repo root:  gpurun -- bash tools/gpu.sh <out> <step> [<step> ...]
# Every step writes under gpurun_out/<out>/ and appends its command line to gpurun_out/<out>/ARGS.txt, which
# the profiles/ index of the round cites.  The first failing step ends the call (no GPU step after a failure).
#
# Steps (arguments after ':' separated by ':'):
#   smoke                    __graft_entry__.smoke()
#   suite                    pytest -m gpu (the whole GPU suite, skip reasons on record)
#   tests:<file>[:<k expr>]  one GPU test file (optionally -k)
#   checked                  the partitioned suites against build/checked/libgossip_hip.so (GOSSIP_EBOUNDS on)
#   checkedall               the whole GPU suite against the checked build
#   evidence                 round 6's bounds evidence: the dense-exchange group tests against the checked build
#                            of round 5's stream kernel (build/checked_unfixed, tools/experiments/
#                            r06_unmasked_stream_entries.patch); failures are the record, not an error
#   bench:<config>[:args]    bench.py --config <config> (args: extra bench flags, '+' for spaces)
#   parts:<P>                bench.py --parts P (config 4 as P vertex blocks on one GPU)
#   rounds:<config>[:t.k=v]  tools/round_profile.py (per-round kernel times; t.key=value tuning)
#   prof:<config>            rocprofv3 kernel trace + stats of the bench command, FETCH_SIZE and WRITE_SIZE passes
#   pmcrounds:<config>[:..]  the same three passes over tools/round_profile.py (tuning args as rounds)
#   ab:<config>:<kernel>:<reps>:<arm>:<arm>...  tools/ab_kernel.py, arms (k=v,k=v or -) alternated in one process
#   libab:<config>:<kernel>:<rounds>:<libA>:<libB>  two builds of libgossip_hip (paths under the repo), one
#                            tools/ab_kernel.py process each, alternated <rounds> times (A B A B ...)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$1; shift
O=gpurun_out/$OUT; mkdir -p $O
log() { echo "$*" >> $O/ARGS.txt; }
fail() { echo "== step $1 failed"; tail -25 "$2"; exit 1; }
PYT="python3 -u -m pytest -x -q -rs --timeout 200 --timeout-method thread"

pmc_summary() {  # $1 dir, $2 label
  python3 tools/pmc_summary.py $1 $1/pmc_summary.json $3 "$2" > /dev/null && python3 -c "
import json; d=json.load(open('$1/pmc_summary.json'))
for k,v in sorted(d['kernels'].items(), key=lambda kv: -kv[1].get('total_ms',0))[:14]:
    print(f\"{k[:48]:48s} n={v.get('launches',0):4d} avg={v.get('avg_ms',0):8.3f} ms  fetch={v.get('fetch_bytes_per_launch_counted',0)/1e9:7.2f} GB  write={v.get('write_bytes_per_launch_counted',0)/1e9:7.2f} GB\")
"
}

for step in "$@"; do
  IFS=: read -r -a a <<< "$step"
  log "$step"
  echo "== $step  ($(date +%H:%M:%S))"
  case ${a[0]} in
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail $step $O/smoke.log
      tail -1 $O/smoke.log ;;
    suite)
      timeout -k 10 1000 $PYT tests -m gpu > $O/pytest.log 2>&1 || fail $step $O/pytest.log
      grep -E "SKIPPED" $O/pytest.log | head -8; tail -1 $O/pytest.log ;;
    tests)
      k=(); [ -n "${a[2]}" ] && k=(-k "${a[2]}")
      f=$O/tests_$(basename ${a[1]} .py).log
      timeout -k 10 900 $PYT "${a[1]}" -m gpu "${k[@]}" > $f 2>&1 || fail $step $f
      tail -1 $f ;;
    checked)
      GOSSIP_HIP_LIB=$PWD/p2p-gossipprotocol_amd/build/checked/libgossip_hip.so timeout -k 10 900 \
        $PYT tests/test_gpu_group.py tests/test_gpu_partitioned.py tests/test_gpu_parity.py -m gpu > $O/checked.log 2>&1 \
        || fail $step $O/checked.log
      tail -1 $O/checked.log ;;
    checkedall)
      GOSSIP_HIP_LIB=$PWD/p2p-gossipprotocol_amd/build/checked/libgossip_hip.so timeout -k 10 1100 \
        $PYT tests -m gpu > $O/checked_all.log 2>&1 || fail $step $O/checked_all.log
      tail -1 $O/checked_all.log ;;
    evidence)
      GOSSIP_HIP_LIB=$PWD/p2p-gossipprotocol_amd/build/checked_unfixed/libgossip_hip.so timeout -k 10 600 \
        python3 -u -m pytest -q -rf --timeout 200 --timeout-method thread tests/test_gpu_group.py -m gpu \
        -k "dense_exchange_forms" > $O/evidence.log 2>&1
      echo "rc=$? (failures expected: GOSSIP_EBOUNDS)"; grep -E "EBOUNDS|index past|passed|failed" $O/evidence.log | cut -c1-300 | head -30 ;;
    bench)
      extra=${a[2]//+/ }
      timeout -k 10 400 python3 -u bench.py --config ${a[1]} $extra > $O/bench_config${a[1]}.json 2> $O/bench_config${a[1]}.err \
        || fail $step $O/bench_config${a[1]}.err
      python3 -c "import json;d=json.loads(open('$O/bench_config${a[1]}.json').read().splitlines()[-1]);r=d['roofline'];print(${a[1]}, d['config']['workload'], d['value'], 'GTEPS', d['ms_per_step'], 'ms', 'frac', r.get('frac'), 'step', r.get('step_frac'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))" ;;
    parts)
      P=${a[1]}
      timeout -k 10 600 python3 -u bench.py --parts $P --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_parts$P.json 2> $O/bench_parts$P.err \
        || fail $step $O/bench_parts$P.err
      python3 -c "import json; d=json.loads(open('$O/bench_parts$P.json').read().splitlines()[-1]); r=d['roofline']; print($P, d['ms_per_step'], d['value'], r.get('frac'), sum(r.get('kernel_ms_per_step').values()), r.get('exchange_ms_per_step'), r.get('exchange_link_ms_per_step'), r.get('projected_ms_per_step'))" ;;
    rounds)
      f=$O/rounds_c${a[1]}$(printf "_%s" "${a[@]:2}").txt
      timeout -k 10 400 python3 -u tools/round_profile.py ${a[1]} "${a[@]:2}" > $f 2>&1 || fail $step $f
      tail -30 $f | cut -c1-220 ;;
    prof)
      C=${a[1]}; d=$O/prof_c$C; mkdir -p $d
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d/c${C}_trace -o run -- python3 -u bench.py --config $C --no-cpu-baseline --steps 5 --warmup 1 > $d/bench_trace.json 2> $d/bench_trace.err || fail $step $d/bench_trace.err
      timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/c${C}_fetch -o run -- python3 -u bench.py --config $C --no-cpu-baseline --no-timing --steps 3 --warmup 1 > $d/bench_fetch.json 2> $d/bench_fetch.err || fail $step $d/bench_fetch.err
      timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/c${C}_write -o run -- python3 -u bench.py --config $C --no-cpu-baseline --no-timing --steps 3 --warmup 1 > $d/bench_write.json 2> $d/bench_write.err || fail $step $d/bench_write.err
      pmc_summary $d "bench.py --config $C (gpu.sh $OUT $step)" c$C
      cut -c1-400 $d/bench_trace.json ;;
    pmcrounds)
      C=${a[1]}; d=$O/pmc_c$C$(printf "_%s" "${a[@]:2}"); mkdir -p $d
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d/c${C}_trace -o run -- python3 -u tools/round_profile.py $C "${a[@]:2}" > $d/trace.txt 2>&1 || fail $step $d/trace.txt
      timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/c${C}_fetch -o run -- python3 -u tools/round_profile.py $C "${a[@]:2}" > $d/fetch.txt 2>&1 || fail $step $d/fetch.txt
      timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/c${C}_write -o run -- python3 -u tools/round_profile.py $C "${a[@]:2}" > $d/write.txt 2>&1 || fail $step $d/write.txt
      pmc_summary $d "round_profile.py $C ${a[*]:2} (gpu.sh $OUT)" c$C ;;
    ab)
      f=$O/ab_c${a[1]}.txt
      timeout -k 10 600 python3 -u tools/ab_kernel.py "${a[@]:1}" > $f 2>&1 || fail $step $f
      tail -20 $f | cut -c1-220 ;;
    libab)
      f=$O/libab_c${a[1]}_${a[2]}.txt
      for ((k = 0; k < ${a[3]}; k++)); do
        for L in "${a[4]}" "${a[5]}"; do
          echo "== $L" >> $f
          GOSSIP_HIP_LIB=$PWD/$L timeout -k 10 300 python3 -u tools/ab_kernel.py ${a[1]} ${a[2]} 3 - >> $f 2>&1 || fail $step $f
        done
      done
      grep -E "^== |median" $f | paste - - | cut -c1-160 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%H:%M:%S)"
