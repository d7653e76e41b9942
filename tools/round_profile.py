"""Per-round kernel times of one config-4 run (after one warm run): frontier
fraction and ms per kernel, cumulative counters differenced per round."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "p2p-gossipprotocol_amd"))
from gossip_hip import Engine  # noqa: E402
from gossip_hip.workloads import config  # noqa: E402

K = ("push_light", "push_heavy", "pull_light", "pull_heavy", "frontier_bits", "bin_scatter", "bin_apply", "inject",
     "liveness", "churn", "kills", "src_count", "rebootstrap", "push_extra", "commit",
     "pb_scatter", "pb_split", "pb_apply", "pull_list", "list_zero", "px_scatter", "compact_send", "apply_remote",
     "heavy_commit")
w = config(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
kw = dict(a.split("=", 1) for a in sys.argv[2:])  # extra engine options, e.g. blocked=off
kw = {k: (int(v) if v.lstrip("-").isdigit() else v) for k, v in kw.items()}
tuning = {k[2:]: kw.pop(k) for k in list(kw) if k.startswith("t.")}  # t.<key>=<int>: gossip_set_tuning
e = Engine(w.n, w.n_msgs, device=0, tuning=tuning, **w.engine_kwargs(), **kw)
e.build_graph()
e.inject(w.origins, w.inject_rounds)
e.run()
e.reset()
e.enable_timing(True)
C = ("#atomics", "#trav", "#heavy_trav", "#pulled", "#gathers", "#needy_rows", "#exit_gathers")
if tuning.get("apply_probe"):  # the streamed apply's phase clocks (100 MHz ticks summed over bins)
    C = C + ("#probe_src", "#probe_init", "#probe_slots", "#probe_finish", "#probe_bins", "#probe_slots_n",
             "#probe_block", "#probe_blocks") + tuple(f"#probe_xcd{x}" for x in range(8))
prev = {k: e.kernel_time(k)[0] for k in K}
prevc = {k: e.kernel_bytes(k) for k in C}
while True:
    st, fin = e.step()
    cur = {k: e.kernel_time(k)[0] for k in K}
    d = {k: round(cur[k] - prev[k], 3) for k in K if cur[k] - prev[k] > 0}
    curc = {k: e.kernel_bytes(k) for k in C}
    dc = {k[1:]: int(curc[k] - prevc[k]) for k in C if curc[k] - prevc[k] > 0}
    extra = ""
    if dc.get("probe_bins"):  # per-bin microseconds of each phase, and the phase's share of 256 CUs' time
        nb = dc["probe_bins"]
        extra = " probe us/bin " + str({k[6:]: round(dc.get(k, 0) / nb / 100, 2)
                                        for k in ("probe_src", "probe_init", "probe_slots", "probe_finish")}) + \
            " ms@256CU " + str({k[6:]: round(dc.get(k, 0) / 1e5 / 256, 3)
                                for k in ("probe_src", "probe_init", "probe_slots", "probe_finish")}) + \
            f" slots/bin {dc.get('probe_slots_n', 0) // nb}" + \
            f" blocks {dc.get('probe_blocks', 0)} block-lifetime ms@256CU {dc.get('probe_block', 0) / 1e5 / 256:.3f}" + \
            " per XCD group ms@32CU " + str([round(dc.get(f"probe_xcd{x}", 0) / 1e5 / 32, 3) for x in range(8)])
        dc = {k: v for k, v in dc.items() if not k.startswith("probe")}
    print(st["round"], f"F={st['frontier'] / w.n:.4f}", d, dc, extra, flush=True)
    prev, prevc = cur, curc
    if fin:
        break
