"""Run one bench.py mode alone (for rocprofv3 kernel traces of a single path).

    python tools/run_mode.py cvrp|slap|slap65k|pomo|dropin|dropin_cvrp|tsp|gen [--k K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode")
    ap.add_argument("--k", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from rl4co_slap_amd import _native

    if os.environ.get("CO_LIB"):  # a variant library (tools/build_variants.sh)
        _native.LIB_PATH = os.environ["CO_LIB"]
    _native.load()
    if a.mode == "cvrp":
        out = bench.bench_cvrp(32768, 100, a.k, 1, 0, dev)
    elif a.mode == "slap":
        out = bench.bench_slap(16384, a.k, 1, 0, dev)
    elif a.mode == "slap65k":
        out = bench.bench_slap(65536, a.k, 1, 0, dev)
    elif a.mode == "steps":
        out = bench.step_kernels_vs_copy(dev)
        out = {k: round(v["kernel_us"], 3) for k, v in out.items()}
    elif a.mode == "dropin":
        out = bench.bench_dropin(65536, 100, a.k, 1, 0, dev)
    elif a.mode == "dropin_cvrp":
        out = bench.bench_dropin_cvrp(32768, 100, a.k, 1, 0, dev)
    elif a.mode == "pomo":
        out = bench.bench_pomo(1024, 100, a.k, 1, 0, dev)
    elif a.mode == "pomo_cert":
        out = bench.bench_pomo(1024, 100, a.k, 1, 0, dev, decode_math="certified")
    elif a.mode == "tsp":
        from rl4co_slap_amd.rollout.engine import TSPFusedEpisode

        import itertools

        n_rot = bench.rotation(65536 * 100 * 16)
        eps = []
        for r in range(n_rot):
            locs, acts = bench.tsp_inputs(65536, 100, 0, salt=r)
            eps.append(TSPFusedEpisode(locs.to(dev), acts.to(dev), policy="teacher", check=True,
                                       layout=os.environ.get("CO_TSP_LAYOUT", "rows")))
        sh = torch.cuda.current_stream(dev).cuda_stream
        cyc = itertools.cycle([e._bound for e in eps])
        wall, ev = bench.timed(lambda: next(cyc)(sh), a.k, 2, 1, dev)
        out = {"launch_us": ev / a.k * 1e6, "wall_us": wall / a.k * 1e6, "batches": n_rot}
    elif a.mode == "gen":
        out = bench.bench_generate_uniform(65536, 100, dev)
    else:
        raise SystemExit(f"unknown mode {a.mode}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
