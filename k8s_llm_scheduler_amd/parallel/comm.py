"""Tensor-parallel process group: one process per GPU, collectives over RCCL (xGMI) or gloo (CPU tests).

On MI355X the backend string ``"nccl"`` IS RCCL.  The decode path issues 2 all-reduces per layer
(row-parallel O and down projections) plus one logits all-gather per step; all of them are
enqueued on the current HIP stream and are captured into the decode hipGraph.

Design choices for 8 x MI355X over point-to-point xGMI (7 links x ~153 GB/s per GPU):
* Decode messages are tiny (B x 8192 bf16 = 16 KiB at B = 1): latency-bound, so the collective
  is issued in-place on the producing tensor (no staging copies) and captured in the graph.
* The vocabulary-parallel LM head gathers fp32 logits [tp, B, V/tp] directly in shard-major
  order; the sampler consumes that layout without a transpose.
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


_DT = {torch.bfloat16: 0, torch.float32: 1, torch.float16: 2, torch.int32: 3}


@dataclass
class TPGroup:
    rank: int = 0
    world: int = 1
    group: Optional[object] = None
    backend: str = "none"
    rccl: Optional[object] = None   # native RcclComm (GPU): graph-capturable collectives
    simulate: bool = False          # shapes of a TP rank, collectives skipped (profiling only)

    @property
    def enabled(self) -> bool:
        return self.world > 1

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1 and not self.simulate:
            if self.rccl is not None and t.is_cuda:
                self.rccl.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], 0, -1)
            elif self.backend == "gloo" and t.dtype == torch.bfloat16:
                f = t.float()
                dist.all_reduce(f, group=self.group)
                t.copy_(f)
            else:
                dist.all_reduce(t, group=self.group)
        return t

    def all_gather_shards(self, t: torch.Tensor) -> torch.Tensor:
        """[..] local -> [world, ..] (shard-major)."""
        if self.world == 1:
            return t.unsqueeze(0)
        if self.simulate:
            return t.unsqueeze(0).expand(self.world, *t.shape).contiguous()
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        t = t.contiguous()
        if self.rccl is not None and t.is_cuda:
            self.rccl.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), _DT[t.dtype], -1)
        elif self.backend == "gloo":
            dist.all_gather(list(out.unbind(0)), t.contiguous(), group=self.group)
        else:
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world > 1:
            dist.broadcast(t, src=src, group=self.group)
        return t

    def barrier(self) -> None:
        if self.world > 1:
            dist.barrier(group=self.group)


class ControlChannel:
    """Rank 0 -> all ranks object broadcast on a CPU (gloo) group: the serving control plane runs
    on rank 0 and every other TP rank follows its engine schedule (engine.LLMEngine._sync)."""

    def __init__(self, rank: int, group=None):
        self.rank = rank
        self.group = group

    def exchange(self, payload):
        obj = [payload]
        dist.broadcast_object_list(obj, src=0, group=self.group)
        return obj[0]


def make_control_channel(tp: TPGroup) -> Optional[ControlChannel]:
    if tp.world <= 1 or tp.simulate:
        return None
    grp = dist.new_group(backend="gloo", timeout=datetime.timedelta(days=7))
    return ControlChannel(tp.rank, grp)


def init_from_env(device_type: Optional[str] = None, timeout_s: int = 600) -> TPGroup:
    """Initialise torch.distributed from torchrun env (RANK/WORLD_SIZE/MASTER_*).  Single
    process when WORLD_SIZE is unset or 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world <= 1:
        return TPGroup()
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    backend = "nccl" if device_type == "cuda" else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", rank))
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    tp = TPGroup(rank, world, dist.group.WORLD, backend)
    if backend == "nccl" and os.environ.get("K8S_TP_COMM", "rccl") == "rccl":
        tp.rccl = make_rccl_comm(tp)
    return tp


def make_rccl_comm(tp: TPGroup):
    """Create the engine's own RCCL communicator (unique id broadcast over torch.distributed)."""
    from .. import ops

    _C = ops.native()
    dev = torch.device("cuda", torch.cuda.current_device())
    uid = torch.zeros(128, dtype=torch.uint8, device=dev)
    if tp.rank == 0:
        uid.copy_(torch.frombuffer(bytearray(_C.RcclComm.unique_id()), dtype=torch.uint8))
    dist.broadcast(uid, src=0, group=tp.group)
    comm = _C.RcclComm(tp.world, tp.rank, bytes(uid.cpu().tolist()))
    # one eager collective so lazy RCCL setup happens outside any graph capture
    probe = torch.ones(16, dtype=torch.float32, device=dev)
    comm.all_reduce(probe.data_ptr(), probe.data_ptr(), probe.numel(), 1, 0, -1)
    torch.cuda.synchronize(dev)
    if float(probe[0]) != float(tp.world):
        raise RuntimeError(f"RCCL communicator self-test failed: {float(probe[0])} != {tp.world}")
    return comm
