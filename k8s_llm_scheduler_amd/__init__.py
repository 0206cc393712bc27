"""MI355X-native LLM-backed Kubernetes scheduler.

Behaviour-compatible with AshishGautamX/K8s-LLM-Scheduler (``scheduler.py`` of the
reference): pods that set ``schedulerName: ai-llama-scheduler`` are watched, the cluster is
snapshotted, a prompt is built, an LLM picks a node and the pod is bound.  The difference is
where the LLM runs: the reference calls the HuggingFace Inference API
(``scheduler.py:425-433``); this package hosts a Llama-3 decision engine in-process on
MI355X GPUs (hand-written gfx950 HIP kernels, RCCL tensor parallelism, hipGraph decode).

Sub-packages
------------
``control``   control plane: config, data model, prompt, cache, breaker, fallback, watch loop
``kube``      Kubernetes API access: in-memory fake, dependency-free REST client
``engine``    decision engine: tokenizer, chat template, paged KV, continuous batching
``models``    Llama-3 graph (8B / 70B / tiny), tensor-parallel sharding, weight init/loading
``ops``       HIP kernels (gfx950) and their torch fp32 reference oracles
``parallel``  tensor-parallel process groups and collectives over RCCL / gloo
``runtime``   native runtime glue: KV block allocator, decode graphs, device memory plans
``utils``     logging, clocks, misc helpers
"""

__version__ = "0.1.0"

SCHEDULER_NAME_DEFAULT = "ai-llama-scheduler"
