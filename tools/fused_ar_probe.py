"""Probe: the fused GEMV all-reduce (gemv.hip GemvAr) at the 70B decode shard shapes, ranks sharing one GPU.
Per shape: error word, wall time, max |error| against the fp32 oracle.  python tools/fused_ar_probe.py W"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from mp_harness import run_ranks  # noqa: E402

SHAPES = [(1, 2048, 512), (2, 2048, 512), (1, 8192, 1024), (2, 8192, 1024), (2, 8192, 512), (2, 4096, 1024),
          (1, 8192, 3584), (2, 8192, 3584), (4, 8192, 1024), (8, 8192, 1024)]


def _rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd import ops
    from k8s_llm_scheduler_amd.parallel import init_from_env

    os.environ["K8S_XGMI_TIMEOUT_S"] = "5"
    tp = init_from_env("cuda", backend="gloo", comm="xgmi")
    comm, dev = tp.xgmi, torch.device("cuda", torch.cuda.current_device())
    out = []
    for i, (M, N, K) in enumerate(SHAPES):
        def operands(r):
            g = torch.Generator(device=dev).manual_seed(7919 * (i + 1) + r)
            x = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, generator=g, device=dev) * (0.5 / K ** 0.5)).to(torch.bfloat16)
            return x, w
        res = torch.randn(M, N, device=dev).to(torch.bfloat16) * 0
        x, w = operands(rank)
        want = res.float()
        for r in range(world):
            xr, wr = operands(r)
            want = want + xr.float() @ wr.float().T
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        y = ops.gemv_allreduce(comm, x, w, res)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        e = comm.error()
        err = float((y.float() - want).abs().max()) if y is not None else None
        bad_rows = [m for m in range(M) if y is not None and float((y[m].float() - want[m]).abs().max()) > 0.05]
        out.append(((M, N, K), e, round(dt, 3), err, bad_rows))
        flag = torch.tensor([1 if e else 0])
        dist.all_reduce(flag)            # (gloo, CPU) every rank resets when any rank timed out: epochs stay equal
        if int(flag):
            comm.reset()
        dist.barrier()
    dist.destroy_process_group()
    return out


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    res = run_ranks(_rank, world, env={"K8S_TP_BACKEND": "gloo", "K8S_TP_COMM": "xgmi"}, timeout_s=300)
    for r in sorted(res):
        for row in res[r]:
            print(f"world {world} rank {r}: shape {row[0]} err_word {row[1]:#x} {row[2]} s max|err| {row[3]} bad rows {row[4]}",
                  flush=True)
