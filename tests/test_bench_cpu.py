"""The bench.py contract the driver depends on (README / task): one JSON line on stdout with the headline metric and
config, here on CPU with the tiny preset; the Poisson-arrival serving mode; and the refusal of prompts that do not fit
--max-model-len (which would otherwise time the fallback path)."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_json_line_contract():
    p = _run("--preset", "tiny", "--steps", "2", "--warmup", "1", "--gen-tokens", "8")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["metric"] == "scheduling_decisions_per_sec" and d["higher_is_better"] is True
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    assert d["dtype"] == "bf16" and "synthetic" in d["data"]
    assert d["config"]["parallelism"] == "tp1" and d["config"]["global_batch"] == 1
    assert abs(d["vs_baseline"] - d["value"] / 0.3) < 0.01 * d["vs_baseline"] + 1e-3


def test_bench_reports_the_timed_workload():
    """with --nodes > 3 every timed step draws a fresh cluster, so the reported prompt / prefill
    sizes must be those of the timed decisions (mean, min, max over the engine requests of the timed region), not one
    pre-timing sample; the prefilled tokens must add up to the engine's own prefill counter."""
    p = _run("--preset", "tiny", "--nodes", "6", "--steps", "3", "--warmup", "1", "--gen-tokens", "4",
             "--max-model-len", "4096")
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    w = d["timed_workload"]
    assert w["engine_requests"] == 3
    pt, pf, gen = w["prompt_tokens"], w["prefilled_tokens"], w["generated_tokens"]
    assert pt["min"] <= pt["mean"] <= pt["max"] and pt["min"] < pt["max"]      # fresh random clusters per step
    assert d["config"]["prompt_tokens"] == pt["mean"]
    assert 0 < pf["min"] and pf["max"] <= pt["max"]
    assert abs(pf["mean"] - d["prefill_tokens_per_decision"]) < 1e-6 * pf["mean"] + 0.11
    assert gen == {"mean": 4, "min": 4, "max": 4}


def test_bench_arrival_mode():
    p = _run("--preset", "tiny", "--arrival-rate", "20", "--steps", "6", "--warmup", "1", "--batch", "4",
             "--gen-tokens", "8")
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["bound"] == 6 and d["config"]["scheduler_mode"] == "continuous"
    assert d["p50_detect_to_bind_ms"] > 0 and set(d["p50_phase_ms"]) == {
        "detect_to_thread", "thread_to_engine_call", "decision_call", "decision_to_bind"}


def test_bench_refuses_prompt_longer_than_max_model_len():
    p = _run("--preset", "tiny", "--nodes", "64", "--max-model-len", "2048", "--steps", "1", "--warmup", "0")
    assert p.returncode != 0 and "max-model-len" in (p.stderr + p.stdout)


def test_bench_arrival_mode_with_replicas():
    """--arrival-rate with --tp < world: 4 ranks as 2 replicas x TP=2 on gloo; rank 0 routes every
    single-pod decision to the least-loaded replica, so both replicas serve pods."""
    from mp_harness import free_port

    env = dict(os.environ, PYTHONPATH=ROOT, K8S_TP_BACKEND="gloo", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "4", "--tp", "2",
           "--preset", "tiny", "--arrival-rate", "20", "--steps", "12", "--warmup", "1", "--batch", "4",
           "--gen-tokens", "8"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert d["bound"] == 12 and d["n_gpus"] == 4 and d["config"]["parallelism"] == "dp2-tp2"
    disp = d["config"]["replica_dispatch"]
    assert sum(disp) == 13 and min(disp) >= 3, disp


def test_bench_self_launches_ranks_for_gpus_n():
    """`python bench.py --gpus N` with no launcher starts the N ranks itself (a
    torch.distributed.run child) and reports N GPUs -- never a 1-rank number labelled N."""
    env = dict(os.environ, PYTHONPATH=ROOT, K8S_TP_BACKEND="gloo", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--tp", "2", "--preset", "tiny",
                        "--steps", "2", "--warmup", "1", "--gen-tokens", "8"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout          # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["config"]["parallelism"] == "dp2-tp2" and d["config"]["global_batch"] == 2
    assert d["scaling"] == "weak" and d["value"] > 0


def test_bench_refuses_gpus_that_disagree_with_world_size():
    env = dict(os.environ, PYTHONPATH=ROOT, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--preset", "tiny",
                        "--steps", "1", "--warmup", "0"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr and not p.stdout.strip()


def test_simulated_tp_reports_the_gpus_it_used():
    """--simulate-tp runs ONE rank's shapes on one device with the collectives skipped; its line
    must not read as a multi-GPU result: n_gpus is the devices used, the simulated degree has its own field."""
    p = _run("--preset", "tiny-tp8", "--simulate-tp", "4", "--steps", "1", "--warmup", "1", "--gen-tokens", "4")
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 1 and d["simulated_tp"] == 4, d
    assert d["config"]["parallelism"] == "tp4-SIMULATED-no-comm"
