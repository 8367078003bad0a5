"""Kubernetes adapter: the seven calls the reference makes through the official C#
``KubernetesClient``, as plain REST over a kubeconfig.

| method                              | REST                                                      | reference call site |
|-------------------------------------|-----------------------------------------------------------|---------------------|
| list_namespaced_pod                 | GET  /api/v1/namespaces/{ns}/pods                         | Agent:86, RAG:202   |
| read_namespaced_pod_log             | GET  /api/v1/namespaces/{ns}/pods/{pod}/log               | Agent:107, RAG:226  |
| list_node                           | GET  /api/v1/nodes                                        | Helpers.cs:91       |
| list_pod_for_all_namespaces         | GET  /api/v1/pods                                         | Helpers.cs:92       |
| list_deployment_for_all_namespaces  | GET  /apis/apps/v1/deployments                            | Helpers.cs:93       |
| read_namespaced_deployment_scale    | GET  /apis/apps/v1/namespaces/{ns}/deployments/{n}/scale  | Agent:133, RAG:284  |
| replace_namespaced_deployment_scale | PUT  same                                                 | Agent:135, RAG:287  |

Errors surface as :class:`K8sApiError` whose message matches the C# SDK's
``HttpOperationException`` ("Operation returned an invalid status code 'NotFound'").
"""
from __future__ import annotations

import base64
import os
import tempfile
from typing import Optional, Protocol

from ..utils.logging import get_logger

log = get_logger("k8s")

_REASONS = {400: "BadRequest", 401: "Unauthorized", 403: "Forbidden", 404: "NotFound", 409: "Conflict",
            422: "UnprocessableEntity", 500: "InternalServerError", 503: "ServiceUnavailable"}


class K8sApiError(RuntimeError):
    def __init__(self, status: int, body: str = ""):
        self.status = status
        self.reason = _REASONS.get(status, str(status))
        self.body = body
        super().__init__(f"Operation returned an invalid status code '{self.reason}'")


class K8sClient(Protocol):
    def list_namespaced_pod(self, namespace: str) -> dict: ...
    def read_namespaced_pod_log(self, name: str, namespace: str, container: Optional[str] = None,
                                tail_lines: Optional[int] = None) -> str: ...
    def list_node(self) -> dict: ...
    def list_pod_for_all_namespaces(self) -> dict: ...
    def list_deployment_for_all_namespaces(self) -> dict: ...
    def read_namespaced_deployment_scale(self, name: str, namespace: str) -> dict: ...
    def replace_namespaced_deployment_scale(self, name: str, namespace: str, body: dict) -> dict: ...


def _materialize(data_b64: Optional[str], path: Optional[str], suffix: str) -> Optional[str]:
    if path:
        return path
    if data_b64:
        f = tempfile.NamedTemporaryFile(delete=False, suffix=suffix)
        f.write(base64.b64decode(data_b64))
        f.close()
        return f.name
    return None


def load_kubeconfig(path: Optional[str] = None, context: Optional[str] = None) -> dict:
    """Parse a kubeconfig (YAML) into {server, token, cert, key, ca, insecure}."""
    import yaml

    path = path or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
    with open(path, "r", encoding="utf-8") as fh:
        kc = yaml.safe_load(fh)
    ctx_name = context or kc.get("current-context")
    ctx = next(c["context"] for c in kc["contexts"] if c["name"] == ctx_name)
    cluster = next(c["cluster"] for c in kc["clusters"] if c["name"] == ctx["cluster"])
    user = next((u["user"] for u in kc.get("users", []) if u["name"] == ctx.get("user")), {}) or {}
    return {
        "server": cluster["server"].rstrip("/"),
        "ca": _materialize(cluster.get("certificate-authority-data"), cluster.get("certificate-authority"), ".crt"),
        "insecure": bool(cluster.get("insecure-skip-tls-verify", False)),
        "token": user.get("token"),
        "cert": _materialize(user.get("client-certificate-data"), user.get("client-certificate"), ".crt"),
        "key": _materialize(user.get("client-key-data"), user.get("client-key"), ".key"),
        "username": user.get("username"),
        "password": user.get("password"),
        "namespace": ctx.get("namespace", "default"),
    }


class RestK8sClient:
    """REST client over httpx (works against a real apiserver or the fake one)."""

    def __init__(self, server: str, token: Optional[str] = None, cert: Optional[str] = None,
                 key: Optional[str] = None, ca: Optional[str] = None, insecure: bool = False,
                 username: Optional[str] = None, password: Optional[str] = None, timeout: float = 30.0,
                 transport=None, **_):
        import httpx

        headers = {"Accept": "application/json"}
        if token:
            headers["Authorization"] = f"Bearer {token}"
        kw = dict(base_url=server, headers=headers, timeout=timeout)
        if transport is not None:
            kw["transport"] = transport
        else:
            kw["verify"] = False if insecure else (ca or True)
            if cert and key:
                kw["cert"] = (cert, key)
        if username and password:
            kw["auth"] = (username, password)
        self.http = httpx.Client(**kw)

    @classmethod
    def from_kubeconfig(cls, path: Optional[str] = None, context: Optional[str] = None):
        return cls(**load_kubeconfig(path, context))

    def _get(self, path: str, params: Optional[dict] = None, text: bool = False):
        r = self.http.get(path, params={k: v for k, v in (params or {}).items() if v is not None})
        if r.status_code >= 300:
            raise K8sApiError(r.status_code, r.text)
        return r.text if text else r.json()

    def list_namespaced_pod(self, namespace: str) -> dict:
        return self._get(f"/api/v1/namespaces/{namespace}/pods")

    def read_namespaced_pod_log(self, name, namespace, container=None, tail_lines=None) -> str:
        return self._get(f"/api/v1/namespaces/{namespace}/pods/{name}/log",
                         {"container": container, "tailLines": tail_lines}, text=True)

    def list_node(self) -> dict:
        return self._get("/api/v1/nodes")

    def list_pod_for_all_namespaces(self) -> dict:
        return self._get("/api/v1/pods")

    def list_deployment_for_all_namespaces(self) -> dict:
        return self._get("/apis/apps/v1/deployments")

    def read_namespaced_deployment_scale(self, name, namespace) -> dict:
        return self._get(f"/apis/apps/v1/namespaces/{namespace}/deployments/{name}/scale")

    def replace_namespaced_deployment_scale(self, name, namespace, body: dict) -> dict:
        r = self.http.put(f"/apis/apps/v1/namespaces/{namespace}/deployments/{name}/scale", json=body)
        if r.status_code >= 300:
            raise K8sApiError(r.status_code, r.text)
        return r.json()


def make_client(cfg=None, fake=None):
    """Real cluster when a kubeconfig is reachable and ``fake_cluster`` is off, else the
    in-memory fake (this environment has no kube-apiserver)."""
    if cfg is not None and not cfg.agent.fake_cluster:
        return RestK8sClient.from_kubeconfig(cfg.agent.kubeconfig if os.path.exists(cfg.agent.kubeconfig) else None)
    from .fake import FakeCluster

    return fake or FakeCluster.default()
