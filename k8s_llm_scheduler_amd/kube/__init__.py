from .api import ApiError, KubeAPI, binding_body, pod_key, pod_uid  # noqa: F401
from .fake import FakeKubeAPI, make_node, make_pod  # noqa: F401
