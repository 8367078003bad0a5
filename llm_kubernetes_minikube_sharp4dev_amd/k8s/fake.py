"""In-memory Kubernetes cluster + a kube-apiserver-shaped HTTP app.

Seeded like the reference's manual fixture (``deployment_test.yaml``: Deployment
``echoserver`` x2 in ``default`` + NodePort Service) plus deployments in the
allow-listed namespaces, a Minikube node, and per-pod logs.  Scaling a deployment
adds / removes pods.  ``fault_rate`` / ``latency_s`` inject failures and delay
(SURVEY §5 fault-injection hook).  Objects use the apiserver's JSON shapes, so
:class:`~.client.RestK8sClient` can talk to :func:`make_apiserver_app` over HTTP.
"""
from __future__ import annotations

import hashlib
import random
import threading
import time
from typing import Optional

import yaml

from .client import K8sApiError


def _clone(o):
    """Copy of a JSON-shaped object (dict / list / scalars): what an apiserver response
    is; ~5x cheaper than copy.deepcopy on the pod objects of the closed-loop benches."""
    if isinstance(o, dict):
        return {k: _clone(v) for k, v in o.items()}
    if isinstance(o, list):
        return [_clone(v) for v in o]
    return o


def _suffix(name: str, i: int) -> str:
    h = hashlib.sha1(f"{name}-{i}".encode()).hexdigest()
    return f"{h[:10]}-{h[10:15]}"


class FakeCluster:
    def __init__(self, node_name: str = "minikube", kubelet: str = "v1.31.0", fault_rate: float = 0.0,
                 latency_s: float = 0.0, seed: int = 0):
        self.lock = threading.RLock()
        self.nodes = [{"metadata": {"name": node_name}, "status": {"nodeInfo": {"kubeletVersion": kubelet}}}]
        self.deployments: dict[tuple[str, str], dict] = {}
        self.pods: dict[tuple[str, str], dict] = {}
        self.logs: dict[tuple[str, str], str] = {}
        self.services: dict[tuple[str, str], dict] = {}
        self.fault_rate = fault_rate
        self.latency_s = latency_s
        self.rng = random.Random(seed)
        self.calls: list[tuple] = []

    # ------------------------------------------------------------ fixtures
    @classmethod
    def default(cls, **kw) -> "FakeCluster":
        c = cls(**kw)
        c.apply_manifest(DEFAULT_MANIFEST)
        for ns, name, n in (("dev", "api", 2), ("staging", "web", 3), ("sharp4dev", "echoserver", 2),
                            ("test-ns-giovanni", "worker", 1), ("kube-system", "coredns", 1)):
            c.create_deployment(ns, name, n, image=f"registry.local/{name}:1.0")
        return c

    def apply_manifest(self, text: str):
        for doc in yaml.safe_load_all(text):
            if not doc:
                continue
            kind = doc.get("kind")
            md = doc.get("metadata", {})
            ns = md.get("namespace", "default")
            if kind == "Deployment":
                spec = doc.get("spec", {})
                ctr = spec.get("template", {}).get("spec", {}).get("containers", [{}])[0]
                self.create_deployment(ns, md["name"], int(spec.get("replicas", 1)), image=ctr.get("image", ""),
                                       container=ctr.get("name", md["name"]))
            elif kind == "Service":
                self.services[(ns, md["name"])] = doc

    def create_deployment(self, ns: str, name: str, replicas: int, image: str = "", container: Optional[str] = None):
        with self.lock:
            self.deployments[(ns, name)] = {
                "metadata": {"name": name, "namespace": ns},
                "spec": {"replicas": replicas, "template": {"spec": {"containers": [
                    {"name": container or name, "image": image}]}}},
                "status": {"replicas": replicas, "readyReplicas": replicas},
            }
            self._reconcile(ns, name)

    def _reconcile(self, ns: str, name: str):
        dep = self.deployments[(ns, name)]
        want = int(dep["spec"]["replicas"] or 0)
        mine = sorted(k for k in self.pods if k[0] == ns and self.pods[k]["metadata"].get("labels", {}).get("app") == name)
        for k in mine[want:]:
            self.pods.pop(k)
            self.logs.pop(k, None)
        ctr = dep["spec"]["template"]["spec"]["containers"][0]["name"]
        have, i = min(len(mine), want), 0
        while have < want:
            pname = f"{name}-{_suffix(name, i)}"
            i += 1
            if (ns, pname) in self.pods:
                continue
            self.pods[(ns, pname)] = {
                "metadata": {"name": pname, "namespace": ns, "labels": {"app": name}},
                "spec": {"nodeName": self.nodes[0]["metadata"]["name"], "containers": [{"name": ctr}]},
                "status": {"phase": "Running"},
            }
            self.logs[(ns, pname)] = None  # generated on first read (a scale to 90 replicas stays cheap)
            have += 1
        dep["status"]["replicas"] = dep["status"]["readyReplicas"] = want

    def _log_text(self, ns: str, pname: str) -> str:
        text = self.logs.get((ns, pname))
        if text is None:
            app = self.pods[(ns, pname)]["metadata"].get("labels", {}).get("app", pname)
            rng = random.Random(f"{ns}/{pname}")
            text = "".join(f"2025-09-17T10:{j // 60:02d}:{j % 60:02d}Z {app} GET /health 200 {rng.randint(1, 40)}ms\n"
                           for j in range(300))
            self.logs[(ns, pname)] = text
        return text

    # ------------------------------------------------------------ fault injection
    def _enter(self, op: str, *args):
        self.calls.append((op,) + args)
        if self.latency_s:
            time.sleep(self.latency_s)
        if self.fault_rate and self.rng.random() < self.fault_rate:
            raise K8sApiError(503, "injected fault")

    # ------------------------------------------------------------ API (K8sClient protocol)
    def list_namespaced_pod(self, namespace: str) -> dict:
        self._enter("list_namespaced_pod", namespace)
        with self.lock:
            return {"kind": "PodList", "items": [_clone(p) for k, p in sorted(self.pods.items()) if k[0] == namespace]}

    def read_namespaced_pod_log(self, name, namespace, container=None, tail_lines=None) -> str:
        self._enter("read_namespaced_pod_log", name, namespace, container, tail_lines)
        with self.lock:
            if (namespace, name) not in self.pods:
                raise K8sApiError(404, f'pods "{name}" not found')
            if container:
                names = [c["name"] for c in self.pods[(namespace, name)]["spec"]["containers"]]
                if container not in names:
                    raise K8sApiError(400, f"container {container} is not valid for pod {name}")
            text = self._log_text(namespace, name) if (namespace, name) in self.logs else ""
        if tail_lines is not None:
            lines = text.splitlines(keepends=True)
            text = "".join(lines[-int(tail_lines):]) if int(tail_lines) > 0 else ""
        return text

    def list_node(self) -> dict:
        self._enter("list_node")
        return {"kind": "NodeList", "items": _clone(self.nodes)}

    def list_pod_for_all_namespaces(self) -> dict:
        self._enter("list_pod_for_all_namespaces")
        with self.lock:
            return {"kind": "PodList", "items": [_clone(p) for _, p in sorted(self.pods.items())]}

    def list_deployment_for_all_namespaces(self) -> dict:
        self._enter("list_deployment_for_all_namespaces")
        with self.lock:
            return {"kind": "DeploymentList", "items": [_clone(d) for _, d in sorted(self.deployments.items())]}

    def read_namespaced_deployment_scale(self, name, namespace) -> dict:
        self._enter("read_namespaced_deployment_scale", name, namespace)
        with self.lock:
            d = self.deployments.get((namespace, name))
            if d is None:
                raise K8sApiError(404, f'deployments.apps "{name}" not found')
            return {"apiVersion": "autoscaling/v1", "kind": "Scale",
                    "metadata": {"name": name, "namespace": namespace},
                    "spec": {"replicas": d["spec"]["replicas"]},
                    "status": {"replicas": d["status"]["replicas"], "selector": f"app={name}"}}

    def replace_namespaced_deployment_scale(self, name, namespace, body: dict) -> dict:
        self._enter("replace_namespaced_deployment_scale", name, namespace)
        with self.lock:
            d = self.deployments.get((namespace, name))
            if d is None:
                raise K8sApiError(404, f'deployments.apps "{name}" not found')
            reps = (body.get("spec") or {}).get("replicas")
            if reps is not None and (not isinstance(reps, int) or reps < 0):
                raise K8sApiError(422, "spec.replicas: Invalid value")
            d["spec"]["replicas"] = reps if reps is not None else 0
            self._reconcile(namespace, name)
        return self.read_namespaced_deployment_scale(name, namespace)


DEFAULT_MANIFEST = """
apiVersion: apps/v1
kind: Deployment
metadata:
  name: echoserver
  labels: {app: echoserver}
spec:
  replicas: 2
  selector: {matchLabels: {app: echoserver}}
  template:
    metadata: {labels: {app: echoserver}}
    spec:
      containers:
      - name: echoserver
        image: gcr.io/google_containers/echoserver:1.10
        ports: [{containerPort: 8080}]
---
apiVersion: v1
kind: Service
metadata: {name: echoserver}
spec:
  type: NodePort
  selector: {app: echoserver}
  ports: [{port: 80, targetPort: 8080, protocol: TCP, nodePort: 30081}]
"""


def make_apiserver_app(cluster: FakeCluster):
    """FastAPI app exposing the fake cluster on the kube-apiserver REST paths."""
    from fastapi import Body, FastAPI, Query
    from fastapi.responses import JSONResponse, PlainTextResponse

    app = FastAPI(title="fake kube-apiserver")

    def err(e: K8sApiError):
        return JSONResponse({"kind": "Status", "status": "Failure", "message": e.body, "reason": e.reason,
                             "code": e.status}, status_code=e.status)

    @app.get("/api/v1/namespaces/{ns}/pods")
    def pods_ns(ns: str):
        return cluster.list_namespaced_pod(ns)

    @app.get("/api/v1/namespaces/{ns}/pods/{name}/log")
    def pod_log(ns: str, name: str, container: Optional[str] = Query(None), tailLines: Optional[int] = Query(None)):
        try:
            return PlainTextResponse(cluster.read_namespaced_pod_log(name, ns, container, tailLines))
        except K8sApiError as e:
            return err(e)

    @app.get("/api/v1/nodes")
    def nodes():
        return cluster.list_node()

    @app.get("/api/v1/pods")
    def pods_all():
        return cluster.list_pod_for_all_namespaces()

    @app.get("/apis/apps/v1/deployments")
    def deps():
        return cluster.list_deployment_for_all_namespaces()

    @app.get("/apis/apps/v1/namespaces/{ns}/deployments/{name}/scale")
    def get_scale(ns: str, name: str):
        try:
            return cluster.read_namespaced_deployment_scale(name, ns)
        except K8sApiError as e:
            return err(e)

    @app.put("/apis/apps/v1/namespaces/{ns}/deployments/{name}/scale")
    def put_scale(ns: str, name: str, body: dict = Body(...)):
        try:
            return cluster.replace_namespaced_deployment_scale(name, ns, body)
        except K8sApiError as e:
            return err(e)

    return app
