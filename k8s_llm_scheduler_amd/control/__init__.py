"""Control plane: behaviour-compatible re-implementation of the reference scheduler loop."""

from .backends import Hang, LocalEngineBackend, ScriptedBackend, first_node_answer  # noqa: F401
from .breaker import CircuitBreaker, CircuitOpenError  # noqa: F401
from .cache import DecisionCache, cache_key  # noqa: F401
from .cluster import ClusterSnapshotter, node_to_metrics, pod_to_spec  # noqa: F401
from .decision import DecisionService, GenerationRequest  # noqa: F401
from .fallback import FallbackPolicy  # noqa: F401
from .jsonextract import extract_json  # noqa: F401
from .models import NodeMetrics, PodSpec, SchedulingDecision  # noqa: F401
from .prompt import PromptEngine  # noqa: F401
from .scheduler import CustomScheduler  # noqa: F401
