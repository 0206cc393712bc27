"""Pod binding (the reference's "Integration Layer", ``scheduler.py:568-620``).

Posts the Binding object of ``scheduler.py:583-595`` to the pod's ``binding`` subresource.  An
API error logs the apiserver's ``message`` and returns False (``:607-615``); any other error
logs and returns False (``:616-620``).
"""

from __future__ import annotations

import json
import logging

from ..kube.api import ApiError, KubeAPI, binding_body

log = logging.getLogger(__name__)


class IntegrationLayer:
    def __init__(self, api: KubeAPI):
        self.api = api

    def bind_pod_to_node(self, pod_name: str, namespace: str, node_name: str) -> bool:
        try:
            self.api.create_binding(namespace, binding_body(pod_name, namespace, node_name))
            log.info(f" Bound pod {namespace}/{pod_name} to node {node_name}")
            return True
        except ApiError as e:
            log.error(f" Error binding pod {pod_name} to node {node_name}: {e}")
            if e.body:
                try:
                    log.error(f"API Error: {json.loads(e.body).get('message', 'No message')}")
                except (json.JSONDecodeError, AttributeError):
                    log.error(f"API Error Body: {e.body}")
            return False
        except Exception as e:  # noqa: BLE001 - reference semantics: never raise out of bind
            log.exception(f" Unexpected error binding pod: {e}")
            return False

    bind = bind_pod_to_node
