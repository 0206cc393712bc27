"""Synthetic cluster-state prompts (benchmarks, tokenizer training, tests).

Prompts are rendered with the real :class:`~k8s_llm_scheduler_amd.control.prompt.PromptEngine`
(the reference template, ``scheduler.py:196-250``) from random but plausible cluster snapshots,
so token counts match what the scheduler sends in production.
"""

from __future__ import annotations

import json
import random
from typing import List, Tuple

from ..control.models import NodeMetrics, PodSpec
from ..control.prompt import PromptEngine

_NAME_SCHEMES = [
    lambda i, r: f"kind-worker{i + 1 if i else ''}",
    lambda i, r: f"minikube-m{i + 1:02d}" if i else "minikube",
    lambda i, r: f"ip-10-0-{r.randint(0, 255)}-{r.randint(1, 254)}.ec2.internal",
    lambda i, r: f"gke-prod-pool-{r.randint(1, 4)}-{r.getrandbits(20):05x}-{r.getrandbits(12):03x}",
    lambda i, r: f"node-{i:02d}",
    lambda i, r: f"worker-{i + 1}",
    lambda i, r: f"aks-nodepool1-{r.randint(10000000, 99999999)}-vmss{i:06d}",
]
_APPS = ["nginx", "redis", "postgres", "api-gateway", "web", "worker", "batch-job", "ml-inference", "kafka",
         "prometheus", "grafana", "frontend", "checkout", "payments", "ai-test-pod"]
_NS = ["default", "prod", "staging", "kube-system", "monitoring", "ml", "data"]
_MEM = ["64Mi", "128Mi", "256Mi", "512Mi", "1Gi", "2Gi", "4Gi", "8Gi"]
_CPU = ["50m", "100m", "250m", "500m", "1", "2", "4"]
_REASONS = [
    "Lowest CPU and memory utilization with ample pod capacity",
    "Node has the most available resources and is Ready",
    "Balances load across the cluster; requests fit comfortably",
    "Least loaded node with sufficient CPU and memory for the request",
    "Fewest running pods and highest free capacity",
]


def random_nodes(rng: random.Random, n: int) -> List[NodeMetrics]:
    scheme = rng.choice(_NAME_SCHEMES)
    out = []
    cpu = rng.choice([2.0, 4.0, 8.0, 16.0, 32.0, 64.0])
    mem = rng.choice([3.84, 7.66, 15.52734375, 31.2, 62.8, 125.6])
    for i in range(n):
        max_pods = rng.choice([110, 110, 250, 58])
        pc = rng.randint(0, max_pods // 2)
        u = pc / max_pods * 50
        out.append(NodeMetrics(scheme(i, rng), u, u, cpu, mem, pc, max_pods, {}, [],
                               [{"type": "Ready", "status": "True", "reason": "KubeletReady"}]))
    return out


def random_pod(rng: random.Random) -> PodSpec:
    from ..control import quantity

    app = rng.choice(_APPS)
    name = f"{app}-{rng.getrandbits(32):08x}"[: rng.randint(len(app) + 3, len(app) + 9)]
    return PodSpec(name, rng.choice(_NS), quantity.pod_cpu(rng.choice(_CPU)), quantity.pod_memory_gb(rng.choice(_MEM)),
                   priority=rng.choice([0, 0, 0, 100, 1000]))


def random_cluster_prompt(rng: random.Random, n_nodes: int) -> Tuple[str, List[NodeMetrics]]:
    nodes = random_nodes(rng, n_nodes)
    return PromptEngine().construct_scheduling_prompt(random_pod(rng), nodes), nodes


def random_answer(rng: random.Random, node: str = "") -> str:
    node = node or _NAME_SCHEMES[rng.randrange(len(_NAME_SCHEMES))](rng.randint(0, 8), rng)
    body = json.dumps({"selected_node": node, "confidence": round(rng.uniform(0.6, 0.98), 2),
                       "reasoning": rng.choice(_REASONS)}, indent=rng.choice([None, 4]))
    return rng.choice(["", "```json\n", "Here is my decision:\n"]) + body + rng.choice(["", "\n```"])


def reference_cluster(n_nodes: int = 3, seed: int = 0) -> Tuple[List[NodeMetrics], List[PodSpec]]:
    """The BASELINE config-1 shape: a kind cluster of `n_nodes` workers (8 cores, ~15.5 GiB) and the
    three ai-test-pods.yaml pods (250m/256Mi, 500m/512Mi, 100m/128Mi)."""
    rng = random.Random(seed)
    nodes = []
    for i in range(n_nodes):
        pc = rng.randint(2, 9)
        u = pc / 110 * 50
        nodes.append(NodeMetrics(f"kind-worker{i + 1 if i else ''}", u, u, 8.0, 15.52734375, pc, 110, {}, [],
                                 [{"type": "Ready", "status": "True", "reason": "KubeletReady"}]))
    pods = [PodSpec("ai-test-pod-1", "default", 0.25, 0.25), PodSpec("ai-test-pod-2", "default", 0.5, 0.5),
            PodSpec("ai-test-pod-3", "default", 0.1, 0.125)]
    return nodes, pods
