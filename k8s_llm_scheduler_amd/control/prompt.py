"""Scheduling prompt construction.

The produced text is byte-identical to the reference ``PromptEngine``
(``scheduler.py:192-252``): system instructions, the pod block, one block per node, the list
of valid names and the closing instruction.  Number formats follow the reference: raw ``str``
of the request floats, ``.1f`` for usage percentages, ``.2f`` for available cores / GB, and
``Status: Ready`` for every node (``scheduler.py:240``) unless
``compat.prompt_status_always_ready`` is switched off, in which case the node's real Ready
condition is printed.

The prompt is assembled from a static prefix (system instructions) and per-request parts so
the engine can prefix-cache the shared system text (long-context row).
"""

from __future__ import annotations

from typing import List, Sequence

from .models import NodeMetrics, PodSpec

# Data contract: the instruction text of scheduler.py:196-214.
SYSTEM_INSTRUCTIONS = "\n".join([
    "You are an intelligent Kubernetes scheduler AI. Your task is to select the BEST ACTUAL "
    "node from the available nodes list for pod placement.",
    "",
    "CRITICAL RULES:",
    '1. You MUST select a node name from the "AVAILABLE NODES" list below',
    "2. The selected_node value MUST be EXACTLY one of the node names",
    "3. Return ONLY valid JSON, nothing else",
    "",
    "Response format:",
    "{",
    '    "selected_node": "node-name",',
    '    "confidence": 0.85,',
    '    "reasoning": "Brief explanation"',
    "}",
    "",
    "Selection criteria:",
    "- Lowest resource utilization (CPU + Memory)",
    "- Available pod capacity",
    "- Resource requests fit available resources",
    "- Node health and readiness",
])


def _pod_block(pod: PodSpec) -> str:
    lines = [
        "",
        "POD TO SCHEDULE:",
        f"Name: {pod.name}",
        f"Namespace: {pod.namespace}",
        f"CPU Request: {pod.cpu_request} cores",
        f"Memory Request: {pod.memory_request} GB",
        f"Priority: {pod.priority}",
        "",
    ]
    return "\n".join(lines)


def _node_block(node: NodeMetrics, status_always_ready: bool) -> str:
    free_cpu = node.available_cpu * (100 - node.cpu_usage_percent) / 100.0
    free_mem = node.available_memory * (100 - node.memory_usage_percent) / 100.0
    status = "Ready" if (status_always_ready or node.is_ready) else "NotReady"
    return "\n".join([
        "",
        f"{node.name}:",
        f"  - CPU Usage: {node.cpu_usage_percent:.1f}% (available: {free_cpu:.2f} cores)",
        f"  - Memory Usage: {node.memory_usage_percent:.1f}% (available: {free_mem:.2f} GB)",
        f"  - Pods: {node.pod_count}/{node.max_pods}",
        f"  - Status: {status}",
        "",
    ])


LAYOUTS = ("reference", "cluster_first")


class PromptEngine:
    """Builds the user prompt for one (pod, cluster snapshot) pair.

    ``layout="reference"`` (default) is byte-identical to the reference: instructions, pod, nodes.
    ``layout="cluster_first"`` (opt-in, ``compat.prompt_layout``) puts the node block before the pod
    block, with the same lines.  Every pod decided against one snapshot then shares the prompt up to
    the pod block, so the engine's prefix cache prefills the cluster state once per batch instead of
    once per pod (long-context row)."""

    def __init__(self, status_always_ready: bool = True, system_instructions: str = SYSTEM_INSTRUCTIONS,
                 layout: str = "reference"):
        if layout not in LAYOUTS:
            raise ValueError(f"prompt layout must be one of {LAYOUTS}, got {layout!r}")
        self.system_prompt = system_instructions
        self.status_always_ready = status_always_ready
        self.layout = layout

    def cluster_block(self, nodes: Sequence[NodeMetrics]) -> str:
        names: List[str] = [n.name for n in nodes]
        body = "".join(_node_block(n, self.status_always_ready) for n in nodes)
        return "AVAILABLE NODES:\n" + body + "\nVALID NODE NAMES: " + ", ".join(names) + "\n"

    def construct_scheduling_prompt(self, pod: PodSpec, nodes: Sequence[NodeMetrics]) -> str:
        names = ", ".join(n.name for n in nodes)
        closing = "\n\nSelect the best node from [" + names + "] and respond with JSON only:"
        if self.layout == "cluster_first":
            return self.system_prompt + "\n\n" + self.cluster_block(nodes) + "\n" + _pod_block(pod) + closing
        return self.system_prompt + "\n\n" + _pod_block(pod) + "\n" + self.cluster_block(nodes) + closing

    # Name used by the rest of this package.
    build = construct_scheduling_prompt
