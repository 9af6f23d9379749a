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


def decode_kernel_us(b, n, dev, flag, reps=100):
    """co_tsp_decode_step (greedy, tanh clip 10) at B x N on a half-visited state, HIP events."""
    from rl4co_slap_amd import _native

    g = torch.Generator().manual_seed(3)
    logits = torch.randn(b, n, generator=g).to(dev)
    mask = (torch.rand(b, n, generator=g) < 0.5).to(dev)
    mask[:, 0] = True
    i = torch.full((b, 1), n // 2, dtype=torch.int64, device=dev)
    first = torch.zeros(b, dtype=torch.int64, device=dev)
    outs = [torch.empty(b, dtype=torch.int64, device=dev), torch.empty(b, device=dev),
            torch.empty((b, n), dtype=torch.bool, device=dev),
            torch.empty((b, 1), dtype=torch.int64, device=dev),
            torch.empty(b, dtype=torch.int64, device=dev),
            torch.empty(b, dtype=torch.bool, device=dev), torch.empty(b, dtype=torch.bool, device=dev)]
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    launch = _native.bind("co_tsp_decode_step", b, n, logits.data_ptr(), n, mask.data_ptr(),
                          10.0, 1.0, flag, None, outs[0].data_ptr(), outs[1].data_ptr(), 0, 0,
                          outs[2].data_ptr(), i.data_ptr(), outs[3].data_ptr(), first.data_ptr(),
                          outs[4].data_ptr(), 0, outs[5].data_ptr(), outs[6].data_ptr(), None,
                          st.data_ptr())
    _, ev = bench.timed(lambda: launch(sh), reps, 5, 1, dev)
    return ev / reps * 1e6


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
    elif a.mode == "dropin_slap":
        out = bench.bench_dropin_slap(16384, a.k, 1, 0, dev)
    elif a.mode == "tsp_chunks":  # teacher-forced stepwise TSP-100 at B = 65,536, chunk sweep
        from rl4co_slap_amd.rollout.engine import TSPStepwiseEpisode

        locs, acts = bench.tsp_inputs(65536, 100, 0)
        locs, acts = locs.to(dev), acts.to(dev)
        out = {}
        for c in (1, 10, 25):
            ep = TSPStepwiseEpisode(locs, acts, chunk=c).capture()
            wall, ev = bench.timed(ep.replay, a.k, 2, 1, dev)
            out[c] = {"us_per_episode": round(wall / a.k * 1e6, 2)}
            del ep
    elif a.mode == "slap_chunks":  # closest-free stepwise SLAP at B = 65,536, chunk sweep
        from rl4co_slap_amd.envs.slap import SLAPGenerator
        from rl4co_slap_amd.rollout.engine import SLAPStepwiseEpisode

        torch.manual_seed(1234)
        td = SLAPGenerator(materialize_dist_mat=False)(65536).to(dev)
        out = {}
        for c in (1, 2, 4, 5, 10, 20):
            ep = SLAPStepwiseEpisode(td, policy="closest", chunk=c).capture()
            wall, ev = bench.timed(ep.replay, a.k, 2, 1, dev)
            byts = bench.slap_chunk_bytes(c) if c > 1 else 234 + 1684 / 20
            out[c] = {"us_per_episode": round(wall / a.k * 1e6, 2),
                      "frac_wall": round(65536 * 20 * byts * a.k / wall / 1e9 / bench.HBM_PEAK_GBS, 4)}
            del ep
    elif a.mode == "slap_decode_kernels":  # the fused SLAP decode step alone, B = 16,384 / 65,536
        out = {b: round(bench.slap_decode_step_kernel_us(b, dev), 3) for b in (16384, 65536)}
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
    elif a.mode == "tsp_nearest":  # the fused nearest-policy episode, TSP-100 B = 65,536
        from rl4co_slap_amd.rollout.engine import TSPFusedEpisode

        locs, _ = bench.tsp_inputs(65536, 100, 0)
        ep = TSPFusedEpisode(locs.to(dev), None, policy="nearest", check=True)
        sh = torch.cuda.current_stream(dev).cuda_stream
        wall, ev = bench.timed(lambda: ep._launch(sh), a.k, 2, 1, dev)
        out = {"ms_per_episode": wall / a.k * 1e3, "launch_ms": ev / a.k * 1e3}
    elif a.mode == "decode_kernels":  # the fused TSP decode step alone, POMO shape, clip 10
        out = {}
        for name, flag in (("certified", _native.DECODE_CERTIFIED), ("fast", _native.DECODE_FAST),
                           ("exact", 0)):
            out[name] = round(decode_kernel_us(102400, 100, dev, flag), 3)
    elif a.mode == "gen":
        out = bench.bench_generate_uniform(65536, 100, dev)
    else:
        raise SystemExit(f"unknown mode {a.mode}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
