"""Spawn N real rank processes (torch.multiprocessing, one process per rank) that run ``fn(rank, world)``
under a torchrun-style environment (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*) and collect each rank's
result or traceback.  Ranks may share one GPU (LOCAL_RANK % device_count) -- the 1-GPU rehearsal of the
8-GPU node -- or each get their own when the GPUs exist."""

import os
import queue
import socket
import sys
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(fn, rank, world, port, env, q, dump_after=None):
    import faulthandler
    import signal

    faulthandler.register(signal.SIGUSR1, all_threads=True)   # the parent asks still-running ranks where they wait
    if dump_after:
        faulthandler.dump_traceback_later(dump_after, exit=False)   # a hung rank shows where it waits
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0", **env)
        q.put((rank, "ok", fn(rank, world)))
    except BaseException:  # noqa: BLE001
        q.put((rank, "fail", traceback.format_exc()))


def run_ranks(fn, world: int, env=None, timeout_s: float = 600.0) -> dict:
    """Returns {rank: result}; raises AssertionError with every failing rank's traceback."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    dump = max(10.0, timeout_s - 30)
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, dict(env or {}), q, dump)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    import time

    t0 = tick = time.monotonic()
    try:
        while len(got) < world and time.monotonic() - t0 < timeout_s:
            if time.monotonic() - tick > 30:   # progress on the real stderr (not captured): long GPU runs stay visible
                tick = time.monotonic()
                print(f"[mp_harness] {fn.__name__}: {len(got)}/{world} ranks done after {tick - t0:.0f}s",
                      file=sys.__stderr__, flush=True)
            try:
                r, status, payload = q.get(timeout=5)
                got[r] = (status, payload)
                if status != "ok":
                    break
            except queue.Empty:
                if any(p.exitcode not in (None, 0) for p in procs):
                    break
    finally:
        if len(got) < world:
            # a rank failed or the run timed out: every rank still running prints its Python stack (all threads) to
            # stderr before it is stopped -- the peer a failed collective waited for shows where it was
            import signal

            for r, p in enumerate(procs):
                if r not in got and p.is_alive():
                    print(f"[mp_harness] {fn.__name__}: rank {r} still running; its stack:", file=sys.__stderr__,
                          flush=True)
                    try:
                        os.kill(p.pid, signal.SIGUSR1)
                    except OSError:
                        pass
                    time.sleep(1.0)
        for p in procs:
            p.join(60 if len(got) == world else 5)
            if p.is_alive():
                p.kill()
    fails = {r: v[1] for r, v in got.items() if v[0] != "ok"}
    assert not fails, "\n".join(f"rank {r}:\n{tb}" for r, tb in fails.items())
    assert len(got) == world, f"ranks finished: {sorted(got)}, exit codes {[p.exitcode for p in procs]}"
    return {r: v[1] for r, v in got.items()}
