"""Data parallelism over decision-engine replicas (BASELINE config 5: "half-node decision engine").

With ``WORLD_SIZE = replicas x tp`` (``engine.tp`` / ``K8S_TP``), ranks ``[r*tp, (r+1)*tp)`` form
replica ``r``: a complete tensor-parallel engine with its own weights, KV cache, RCCL communicator and
xGMI peer regions (``comm.init_from_env``).  Global rank 0 runs the control plane (the reference's
whole ``scheduler.py``) and the leader of replica 0.  The leader of every other replica receives
batches of chat requests from rank 0 over a two-rank gloo link, runs them on its engine (its TP
followers track its schedule through the replica's ``ControlChannel``) and sends the completion
texts back.

:class:`ReplicaRouterBackend` is the decision backend on rank 0: a batch (``scheduler.mode:
batched``) is dealt round-robin over the replicas, remote shares go out on one thread per link
while the local share runs on rank 0's own engine, and the texts come back in request order.  A
failure of any share raises, so retries / circuit breaker / fallback of the decision service see
one failed engine call, as for a single engine.  The reference has no counterpart (one remote
HTTPS call per pod, ``scheduler.py:425-433``).
"""

from __future__ import annotations

import datetime
import logging
import threading
from typing import List, Optional, Sequence

import torch.distributed as dist

from .comm import TPGroup

log = logging.getLogger(__name__)

_STOP = "__stop__"


class ReplicaLink:
    """Two-rank gloo group between global rank 0 and the leader of one remote replica."""

    def __init__(self, replica: int, leader: int, group):
        self.replica = replica
        self.leader = leader        # global rank of the remote replica's TP rank 0
        self.group = group
        self._lock = threading.Lock()

    def _bcast(self, obj, src: int):
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.group)
        return box[0]

    # rank-0 side
    def request(self, payload):
        with self._lock:   # one outstanding batch per link: request/reply stay paired
            self._bcast(payload, 0)
            return self._bcast(None, self.leader)

    def stop(self) -> None:
        with self._lock:
            self._bcast(_STOP, 0)

    # leader side
    def receive(self):
        return self._bcast(None, 0)

    def reply(self, payload) -> None:
        self._bcast(payload, self.leader)


def make_replica_links(tp: TPGroup) -> List[ReplicaLink]:
    """Collective over the world (every rank must call it).  Rank 0 gets one link per remote
    replica, a remote leader gets its own link, every other rank an empty list."""
    links: List[ReplicaLink] = []
    if tp.replicas <= 1 or tp.simulate:
        return links
    me = tp.global_rank
    for r in range(1, tp.replicas):
        leader = r * tp.world
        g = dist.new_group(ranks=[0, leader], backend="gloo", timeout=datetime.timedelta(days=7))
        if me in (0, leader):
            links.append(ReplicaLink(r, leader, g))
    return links


class ReplicaRouterBackend:
    """Decision backend of rank 0 that spreads every batch over all engine replicas."""

    def __init__(self, local, links: Sequence[ReplicaLink]):
        self.local = local
        self.links = list(links)
        self.name = f"{getattr(local, 'name', 'local')}x{len(self.links) + 1}"
        self.dispatched = [0] * (len(self.links) + 1)

    @property
    def replicas(self) -> int:
        return len(self.links) + 1

    def complete(self, requests) -> List[str]:
        n = self.replicas
        shares = [list(requests[i::n]) for i in range(n)]
        results: List[Optional[List[str]]] = [None] * n
        errors: List[Optional[BaseException]] = [None] * n

        def remote(i: int) -> None:
            try:
                resp = self.links[i - 1].request({"requests": shares[i]})
                if "error" in resp:
                    raise RuntimeError(f"replica {i}: {resp['error']}")
                results[i] = list(resp["texts"])
            except BaseException as e:  # noqa: BLE001 -- re-raised on the calling thread
                errors[i] = e

        threads = [threading.Thread(target=remote, args=(i,), daemon=True) for i in range(1, n) if shares[i]]
        for t in threads:
            t.start()
        try:
            results[0] = self.local.complete(shares[0]) if shares[0] else []
        except BaseException as e:  # noqa: BLE001
            errors[0] = e
        for t in threads:
            t.join()
        for i in range(n):
            self.dispatched[i] += len(shares[i])
            if shares[i] and errors[i] is not None:
                raise errors[i]
        out: List[str] = [""] * len(requests)
        for i in range(n):
            for j, text in enumerate(results[i] or []):
                out[i + j * n] = text
        return out

    def shutdown(self) -> None:
        for link in self.links:
            try:
                link.stop()
            except Exception as e:  # noqa: BLE001
                log.warning(f" replica {link.replica} did not acknowledge shutdown: {e}")


def serve_replica(backend, link: ReplicaLink, engine=None) -> None:
    """Leader of a remote replica: answer rank 0's batches until it sends stop, then release the
    replica's TP followers (``engine.shutdown_workers``)."""
    try:
        while True:
            msg = link.receive()
            if msg == _STOP:
                return
            try:
                texts = backend.complete(msg["requests"])
                link.reply({"texts": texts})
            except Exception as e:  # noqa: BLE001 -- reported to rank 0, which decides (retry/fallback)
                link.reply({"error": f"{type(e).__name__}: {e}"})
    finally:
        if engine is not None:
            engine.shutdown_workers()
