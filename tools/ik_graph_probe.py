"""IK leg launch overhead: K back-to-back pnp_ik_dls calls (4096 solves each) issued directly,
as one captured HIP graph replayed per call, and as one graph holding all K calls; prints the
wall time per call and the kernel's own duration (HIP events around one call)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
import bench  # noqa: E402
from pnp_amd import workloads  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402


def main():
    K = 50
    torch.cuda.set_device(0)
    eng = get_engine()
    B = 4096
    q0, tgt, _, _ = bench.ik_inputs(eng, eng.model, 0, B, "waypoint")
    prm = workloads.IK_PARAMS["default"]
    dev = eng.device
    out = dict(q=torch.empty(B, 7, device=dev), final_pos=torch.empty(B, 3, device=dev),
               pos_error=torch.empty(B, device=dev), iterations=torch.empty(B, dtype=torch.int32, device=dev),
               flags=torch.empty(B, dtype=torch.uint8, device=dev))
    call = lambda: eng.ik_dls_into(q0, tgt, out, **prm)
    for _ in range(5):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); call(); e1.record(); torch.cuda.synchronize()
    print(f"kernel (one call, events): {e0.elapsed_time(e1) * 1e3:.1f} us", flush=True)
    t = time.perf_counter()
    for _ in range(K):
        call()
    torch.cuda.synchronize()
    print(f"direct: {(time.perf_counter() - t) / K * 1e6:.1f} us per call", flush=True)
    t = time.perf_counter()
    for _ in range(K):
        call()
    print(f"direct, host side only: {(time.perf_counter() - t) / K * 1e6:.1f} us per call", flush=True)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        call()
        torch.cuda.synchronize()
        with torch.cuda.graph(g1, stream=s):
            call()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(K):
        g1.replay()
    torch.cuda.synchronize()
    print(f"graph of 1 call, replayed: {(time.perf_counter() - t) / K * 1e6:.1f} us per call", flush=True)
    gk = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(gk, stream=s):
            for _ in range(K):
                call()
    torch.cuda.synchronize()
    t = time.perf_counter()
    gk.replay()
    torch.cuda.synchronize()
    print(f"graph of {K} calls: {(time.perf_counter() - t) / K * 1e6:.1f} us per call", flush=True)
    t = time.perf_counter()
    gk.replay()
    torch.cuda.synchronize()
    print(f"graph of {K} calls (again): {(time.perf_counter() - t) / K * 1e6:.1f} us per call", flush=True)


if __name__ == "__main__":
    main()
