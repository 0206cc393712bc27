"""Bounded start-up stages (utils/stages.py): every stage of bringing the engine up is timed, and a
stage that outlives its bound ends the process with exit code 3 and a line naming the stage and the rank -- the
first real multi-GPU run must fail loudly and say where, not hang until the driver's timeout."""

import json
import os
import subprocess
import sys

import pytest

from k8s_llm_scheduler_amd.utils import stages

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", sorted(stages.DEFAULT_BOUNDS))
def test_every_stage_times_out_with_its_name(name):
    code = ("import os; from k8s_llm_scheduler_amd.utils import stages; stages.install(rank=5)\n"
            f"with stages.stage({name!r}):\n    pass\nprint('not reached')")
    env = dict(os.environ, PYTHONPATH=ROOT, K8S_STALL_STAGE=name, K8S_STALL_S="30",
               **{f"K8S_STAGE_TIMEOUT_{name.upper()}": "0.3"})
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode == stages.EXIT_CODE, (p.returncode, p.stderr)
    assert f"stage '{name}'" in p.stderr and "rank 5" in p.stderr and "not reached" not in p.stdout


def test_stages_record_times_without_a_watch():
    with stages.stage("unit_a"):
        pass
    with stages.stage("unit_a"):
        pass
    t = stages.timings()
    assert "unit_a" in t and t["unit_a"] >= 0.0


def _bench(*args, env=None, timeout=300):
    e = dict(os.environ, PYTHONPATH=ROOT, **(env or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_reports_init_stages_and_exits_on_a_stalled_stage():
    ok = _bench("--preset", "tiny", "--steps", "1", "--warmup", "1", "--gen-tokens", "4")
    assert ok.returncode == 0, ok.stderr[-2000:]
    d = json.loads(ok.stdout.strip().splitlines()[-1])
    assert {"engine_build", "graph_capture", "warmup"} <= set(d["init_stages"]["rank0"])
    assert "allreduce_transports" in d
    bad = _bench("--preset", "tiny", "--steps", "1", "--warmup", "1", "--gen-tokens", "4",
                 env={"K8S_STALL_STAGE": "warmup", "K8S_STALL_S": "60", "K8S_STAGE_TIMEOUT_WARMUP": "1"})
    assert bad.returncode == stages.EXIT_CODE and "stage 'warmup'" in bad.stderr and not bad.stdout.strip()


def test_two_rank_bench_reports_the_slowest_rank_and_fails_on_a_stalled_process_group():
    """gloo, 2 ranks (self-launched): the JSON carries rank 0's stage times and the slowest rank per stage; a rank
    whose process-group stage stalls makes the whole job exit non-zero with the stage named."""
    env = {"K8S_TP_BACKEND": "gloo", "OMP_NUM_THREADS": "1"}
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        os.environ.pop(k, None)
    ok = _bench("--gpus", "2", "--preset", "tiny", "--steps", "1", "--warmup", "1", "--gen-tokens", "4", env=env,
                timeout=400)
    assert ok.returncode == 0, ok.stderr[-3000:]
    d = json.loads([l for l in ok.stdout.splitlines() if l.startswith("{")][-1])
    st = d["init_stages"]
    assert "process_group" in st["rank0"] and st["slowest"]["process_group"]["rank"] in (0, 1)
    assert any(k.startswith("prefill:gloo:") or k.startswith("decode:gloo:") for k in d["allreduce_transports"])
    bad = _bench("--gpus", "2", "--preset", "tiny", "--steps", "1", "--warmup", "1", "--gen-tokens", "4",
                 env=dict(env, K8S_STALL_STAGE="process_group", K8S_STALL_S="120",
                          K8S_STAGE_TIMEOUT_PROCESS_GROUP="2"), timeout=400)
    assert bad.returncode != 0 and "stage 'process_group'" in bad.stderr
