"""RCCL communicator of the engine (world size 1 on the single-GPU test box): collectives on the
current stream, and captured + replayed inside a hipGraph (the decode-step pattern).  Multi-rank
correctness of the TP model is covered on CPU by test_tp_gloo.py."""

import pytest
import torch

from k8s_llm_scheduler_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    C = ops.native()
    return C.RcclComm(1, 0, C.RcclComm.unique_id())


def test_allreduce_allgather(comm):
    x = torch.randn(8192, device="cuda").bfloat16()
    y = x.clone()
    comm.all_reduce(y.data_ptr(), y.data_ptr(), y.numel(), 0, 0, -1)
    torch.testing.assert_close(y, x)
    out = torch.empty(1, 100, device="cuda")
    src = torch.randn(100, device="cuda")
    comm.all_gather(src.data_ptr(), out.data_ptr(), 100, 1, -1)
    torch.testing.assert_close(out[0], src)


def test_collective_in_hipgraph(comm):
    buf = torch.zeros(4096, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        buf.add_(1)
        comm.all_reduce(buf.data_ptr(), buf.data_ptr(), buf.numel(), 0, 0, -1)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        buf.add_(1)
        comm.all_reduce(buf.data_ptr(), buf.data_ptr(), buf.numel(), 0, 0, -1)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert float(buf[0]) == 4.0
