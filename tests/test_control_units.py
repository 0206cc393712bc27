"""T1 unit tests of the control plane: config precedence, quantity parsing,
golden prompt, cache TTL/FIFO, breaker state machine, JSON extraction, fallback strategies."""

import json

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from k8s_llm_scheduler_amd.config import load_config, load_dotenv
from k8s_llm_scheduler_amd.control import quantity
from k8s_llm_scheduler_amd.control.breaker import CLOSED, HALF_OPEN, OPEN, CircuitBreaker, CircuitOpenError
from k8s_llm_scheduler_amd.control.cache import DecisionCache, cache_key
from k8s_llm_scheduler_amd.control.fallback import FallbackPolicy
from k8s_llm_scheduler_amd.control.jsonextract import extract_json, json_object_closed
from k8s_llm_scheduler_amd.control.models import NodeMetrics, PodSpec, SchedulingDecision
from k8s_llm_scheduler_amd.control.prompt import PromptEngine


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def mk_nodes(pods, ready=None, max_pods=110):
    out = []
    for i, pc in enumerate(pods):
        u = pc / max_pods * 50 if max_pods else 0
        ok = True if ready is None else ready[i]
        out.append(NodeMetrics(f"kind-worker{i + 1 if i else ''}", u, u, 8.0, 15.52734375, pc, max_pods, {}, [],
                               [{"type": "Ready", "status": "True" if ok else "False", "reason": ""}]))
    return out


# ------------------------------------------------------------------ config
def test_config_defaults_and_precedence(tmp_path):
    y = tmp_path / "config.yaml"
    y.write_text("scheduler:\n  name: from-yaml\nllm:\n  max_retries: 7\n  temperature: 0.5\n"
                 "cache:\n  ttl: 10\nfallback:\n  strategy: least_loaded\n")
    cfg = load_config(y, environ={})
    assert cfg.scheduler.name == "from-yaml" and cfg.llm.max_retries == 7 and cfg.llm.temperature == 0.5
    assert cfg.cache.ttl == 10.0 and cfg.fallback.strategy == "least_loaded"
    assert cfg.circuit_breaker.failure_threshold == 5 and cfg.llm.max_tokens == 200  # defaults
    cfg = load_config(y, environ={"SCHEDULER_NAME": "from-env", "LLM_MAX_RETRIES": "2", "CACHE_TTL": "3"})
    assert cfg.scheduler.name == "from-env" and cfg.llm.max_retries == 2 and cfg.cache.ttl == 3.0
    cfg = load_config(tmp_path / "missing.yaml", environ={})
    assert cfg.scheduler.name == "ai-llama-scheduler" and cfg.source is None


def test_repo_config_yaml_is_reference_compatible():
    cfg = load_config("config.yaml", environ={})
    assert cfg.scheduler.name == "ai-llama-scheduler"
    assert cfg.llm.model == "meta-llama/Llama-3.3-70B-Instruct"
    assert (cfg.llm.max_retries, cfg.llm.temperature, cfg.llm.max_tokens) == (3, 0.3, 200)
    assert (cfg.cache.enabled, cfg.cache.ttl, cfg.cache.max_size) == (True, 300, 100)
    assert cfg.fallback.strategy == "resource_balanced"
    assert (cfg.circuit_breaker.failure_threshold, cfg.circuit_breaker.timeout) == (5, 60)


def test_dotenv(tmp_path):
    p = tmp_path / ".env"
    p.write_text("# c\nA=1\nexport B='two'\nC=\"3\"  \nD=x # trailing\n")
    env = {"A": "keep"}
    got = load_dotenv(p, env)
    assert got == {"A": "1", "B": "two", "C": "3", "D": "x"}
    assert env["A"] == "keep" and env["B"] == "two"


# ------------------------------------------------------------------ quantities
@pytest.mark.parametrize("s,cores", [("250m", 0.25), ("2", 2.0), ("0.5", 0.5), ("1500m", 1.5)])
def test_cpu_parse_agrees(s, cores):
    assert quantity.node_cpu(s, "reference") == cores == quantity.node_cpu(s, "full")


@pytest.mark.parametrize("s", ["16393220Ki", "512Mi", "8Gi", "1073741824"])
def test_node_memory_bit_identical(s):
    assert quantity.node_memory_gb(s, "reference") == quantity.node_memory_gb(s, "full")


def test_reference_quirks():
    with pytest.raises(ValueError):
        quantity.node_cpu("100n", "reference")
    with pytest.raises(ValueError):
        quantity.node_memory_gb("1G", "reference")
    assert quantity.pod_memory_gb("1G", "reference") == 0.0       # quirk 12: pod side -> 0
    assert quantity.pod_memory_gb("1073741824", "reference") == 0.0
    assert quantity.node_cpu("100n", "full") == pytest.approx(1e-7)
    assert quantity.node_memory_gb("1G", "full") == pytest.approx(1e9 / 2 ** 30)
    assert quantity.pod_memory_gb("256Mi", "full") == 0.25


# ------------------------------------------------------------------ prompt (golden, generated from the reference code)
def test_golden_prompt_3_nodes(fixtures_dir):
    pod = PodSpec("ai-test-pod-1", "default", 0.25, 0.25, {}, [], {}, 0)
    got = PromptEngine().construct_scheduling_prompt(pod, mk_nodes([4, 7, 2]))
    assert got == (fixtures_dir / "golden_prompt_3nodes.txt").read_text()


def test_golden_prompt_1_node(fixtures_dir):
    pod = PodSpec("web", "prod", 1.5, 0.0, {}, [], {}, 1000)
    got = PromptEngine().construct_scheduling_prompt(pod, mk_nodes([0]))
    assert got == (fixtures_dir / "golden_prompt_1node.txt").read_text()


def test_prompt_status_quirk_switch():
    nodes = mk_nodes([1, 2], ready=[True, False])
    pod = PodSpec("p", "d", 0.1, 0.1)
    assert "Status: NotReady" not in PromptEngine(True).build(pod, nodes)
    assert "Status: NotReady" in PromptEngine(False).build(pod, nodes)


# ------------------------------------------------------------------ cache
def test_cache_ttl_and_fifo():
    clk = Clock()
    c = DecisionCache(ttl=300, max_size=2, clock=clk)
    nodes = mk_nodes([1, 2])
    pods = [PodSpec(f"p{i}", "d", 0.1 * (i + 1), 0.1, priority=0) for i in range(3)]
    d = [SchedulingDecision(f"n{i}", 0.9, "r") for i in range(3)]
    c.set(pods[0], nodes, d[0])
    clk.t += 1
    c.set(pods[1], nodes, d[1])
    assert c.get(pods[0], nodes) is d[0]          # get does not refresh (FIFO, not LRU)
    clk.t += 1
    c.set(pods[2], nodes, d[2])                   # evicts the oldest insertion: pods[0]
    assert c.get(pods[0], nodes) is None and c.get(pods[1], nodes) is d[1]
    clk.t += 300
    assert c.get(pods[1], nodes) is None          # expired (lazily deleted)
    assert len(c) == 1


def test_cache_key_ignores_pod_identity():
    nodes = mk_nodes([1, 2])
    a = PodSpec("a", "ns1", 0.25, 0.25)
    b = PodSpec("b", "ns2", 0.25, 0.25)
    assert cache_key(a, nodes) == cache_key(b, list(reversed(nodes)))   # quirk 5 + sorted nodes
    assert cache_key(a, nodes) != cache_key(PodSpec("a", "ns1", 0.5, 0.25), nodes)


# ------------------------------------------------------------------ breaker
def _boom():
    raise RuntimeError("x")


def test_breaker_state_machine():
    clk = Clock()
    b = CircuitBreaker(failure_threshold=3, timeout=60, clock=clk)
    for _ in range(2):
        with pytest.raises(RuntimeError):
            b.call(_boom)
        assert b.call(lambda: 1) == 1              # success in CLOSED does not reset (quirk 6)
    assert b.failures == 2 and b.state == CLOSED
    with pytest.raises(RuntimeError):
        b.call(_boom)
    assert b.state == OPEN
    with pytest.raises(CircuitOpenError, match="Circuit breaker is OPEN"):
        b.call(lambda: 1)
    clk.t += 61
    with pytest.raises(RuntimeError):
        b.call(_boom)                              # HALF_OPEN trial fails -> OPEN again
    assert b.state == OPEN
    clk.t += 61
    assert b.call(lambda: 2) == 2 and b.state == CLOSED and b.failures == 0
    assert b.state != HALF_OPEN


def test_breaker_reset_on_success_when_fixed():
    b = CircuitBreaker(failure_threshold=2, cumulative_failures=False)
    with pytest.raises(RuntimeError):
        b.call(_boom)
    b.call(lambda: 0)
    with pytest.raises(RuntimeError):
        b.call(_boom)
    assert b.state == CLOSED


# ------------------------------------------------------------------ json extraction
def test_extract_json_strategies():
    assert extract_json('x ```json\n{"a": 1}\n``` y') == {"a": 1}
    assert extract_json('{"a": 1} then {"b": 2}') == {"b": 2}          # last object wins
    assert extract_json('{"a": {"b": 2}}') == {"b": 2}                  # rfind('{') = inner object
    assert extract_json('{"a": 1, "r": "}"} {bad') == {"a": 1, "r": "}"} or extract_json('{"a": 1, "r": "}"} {bad') is None
    assert extract_json("no json") is None
    assert extract_json('```json\nnot json\n``` {"c": 3}') == {"c": 3}
    assert json_object_closed('pre {"a": {"b": 1}}') and not json_object_closed('{"a": {')


@settings(max_examples=200, deadline=None)
@given(st.dictionaries(st.text(min_size=1, max_size=8), st.one_of(st.integers(), st.text(max_size=8)),
                       min_size=1, max_size=4), st.text(max_size=20).filter(lambda s: "{" not in s and "}" not in s))
def test_extract_json_roundtrip(obj, noise):
    text = json.dumps(obj)
    if "{" in text[1:] or "}" in text[:-1]:
        return  # braces inside strings defeat the naive counter (reference behaviour)
    assert extract_json(noise + text + noise) == obj


# ------------------------------------------------------------------ fallback
def test_fallback_resource_balanced_and_ready_filter():
    nodes = mk_nodes([10, 2, 1], ready=[True, True, False])
    d = FallbackPolicy("resource_balanced").decide(nodes, "why")
    assert d == SchedulingDecision("kind-worker2", 0.4, "Fallback (resource_balanced): why", True)


def test_fallback_least_loaded_ties_keep_first():
    nodes = mk_nodes([3, 3])
    assert FallbackPolicy("least_loaded").decide(nodes, "r").selected_node == "kind-worker"


def test_fallback_round_robin_quirk():
    nodes = mk_nodes([1, 9, 4])
    assert FallbackPolicy("round_robin").decide(nodes, "r").selected_node == "kind-worker2"   # MOST pods
    assert FallbackPolicy("whatever").decide(nodes, "r").selected_node == "kind-worker2"
    rr = FallbackPolicy("round_robin", round_robin_picks_most_pods=False)
    assert [rr.decide(nodes, "r").selected_node for _ in range(4)] == \
        ["kind-worker", "kind-worker2", "kind-worker3", "kind-worker"]


def test_fallback_edge_cases():
    assert FallbackPolicy().decide([], "r") == SchedulingDecision("", 0.0, "No nodes available", True)
    d = FallbackPolicy().decide(mk_nodes([1], ready=[False]), "r")
    assert d == SchedulingDecision("", 0.0, "Fallback failed: r", True)
    assert FallbackPolicy().decide(mk_nodes([0], max_pods=0), "r").selected_node == "kind-worker"


def test_cluster_first_layout_same_lines_shared_prefix():
    from k8s_llm_scheduler_amd.control.prompt import PromptEngine

    nodes = mk_nodes([4, 7, 2])
    pods = [PodSpec(f"p{i}", "default", 0.25 * (i + 1), 0.5, {}, [], {}, 0) for i in range(2)]
    ref_pe, cf_pe = PromptEngine(), PromptEngine(layout="cluster_first")
    a, b = (cf_pe.build(p, nodes) for p in pods)
    assert sorted(a.splitlines()) == sorted(ref_pe.build(pods[0], nodes).splitlines())
    shared = len(cf_pe.system_prompt) + len(cf_pe.cluster_block(nodes))
    assert a[:shared] == b[:shared] and a != b
    with pytest.raises(ValueError):
        PromptEngine(layout="bogus")


def test_reference_config_yaml_logging_section_stays_inert(tmp_path):
    """the reference's own config.yaml (logging.format json, file scheduler.log) must not switch
    on JSON file logging -- the reference never read that section (scheduler.py:27-28)."""
    from k8s_llm_scheduler_amd.config import load_config

    ref = tmp_path / "config.yaml"
    ref.write_text("logging:\n  level: DEBUG\n  format: json\n  file: scheduler.log\n")
    cfg = load_config(ref, environ={})
    assert (cfg.logging.level, cfg.logging.format, cfg.logging.file) == ("INFO", "text", None)
    ours = tmp_path / "ours.yaml"
    ours.write_text("compat:\n  yaml_logging: true\nlogging:\n  format: json\n  file: s.log\n")
    cfg = load_config(ours, environ={})
    assert (cfg.logging.format, cfg.logging.file) == ("json", "s.log")
    assert load_config(ours, environ={"LOG_FORMAT": "text"}).logging.format == "text"
