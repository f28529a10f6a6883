"""Minimal Kubernetes REST client (stdlib only).

Reference: pkg/util/client/client.go:17-42 (in-cluster config, else
$KUBECONFIG) and the client-go calls the reference makes: node
GET/LIST/UPDATE/PATCH, pod GET/LIST/PATCH/bind (pkg/util/util.go:238-294,
pkg/scheduler/scheduler.go:312-352).  Differences: pod listing for a node uses
a `spec.nodeName` field selector instead of listing every pod in the cluster
(reference util.go:41-66).
"""
from __future__ import annotations

import base64
import json
import os
import ssl
import tempfile
import threading
import urllib.error
import urllib.parse
import urllib.request

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class ApiError(Exception):
    def __init__(self, status: int, body: str = ""):
        super().__init__(f"HTTP {status}: {body[:300]}")
        self.status = status
        self.body = body


class KubeClient:
    def __init__(self, server: str, token: str | None = None, ca_file: str | None = None,
                 cert_file: str | None = None, key_file: str | None = None,
                 insecure: bool = False, timeout: float = 10.0):
        self.server = server.rstrip("/")
        self.token = token
        self.timeout = timeout
        self._lock = threading.Lock()
        if self.server.startswith("https"):
            ctx = ssl.create_default_context(cafile=ca_file) if ca_file else ssl.create_default_context()
            if insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            if cert_file:
                ctx.load_cert_chain(cert_file, key_file)
            self._ctx = ctx
        else:
            self._ctx = None

    # ---- construction ------------------------------------------------------------
    @classmethod
    def from_env(cls) -> "KubeClient":
        host = os.environ.get("KUBERNETES_SERVICE_HOST")
        if host and os.path.exists(f"{SA_DIR}/token"):
            port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            token = open(f"{SA_DIR}/token").read().strip()
            return cls(f"https://{host}:{port}", token=token, ca_file=f"{SA_DIR}/ca.crt")
        kc = os.environ.get("KUBECONFIG", os.path.expanduser("~/.kube/config"))
        if os.path.exists(kc):
            return cls.from_kubeconfig(kc)
        url = os.environ.get("VGPU_APISERVER")
        if url:
            return cls(url, token=os.environ.get("VGPU_APISERVER_TOKEN"))
        raise RuntimeError("no in-cluster config, KUBECONFIG or VGPU_APISERVER")

    @classmethod
    def from_kubeconfig(cls, path: str) -> "KubeClient":
        import yaml
        cfg = yaml.safe_load(open(path))
        cur = cfg.get("current-context")
        ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == cur)
        cl = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in cfg.get("users", []) if u["name"] == ctx.get("user")), {})

        def materialize(data_key, file_key, src):
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                f = tempfile.NamedTemporaryFile(delete=False, suffix=".pem")
                f.write(base64.b64decode(src[data_key]))
                f.close()
                return f.name
            return None

        return cls(cl["server"], token=user.get("token"),
                   ca_file=materialize("certificate-authority-data", "certificate-authority", cl),
                   cert_file=materialize("client-certificate-data", "client-certificate", user),
                   key_file=materialize("client-key-data", "client-key", user),
                   insecure=bool(cl.get("insecure-skip-tls-verify")))

    # ---- transport -----------------------------------------------------------------
    def request(self, method: str, path: str, body=None, content_type: str = "application/json",
                query: dict | None = None):
        url = self.server + path
        if query:
            url += "?" + urllib.parse.urlencode(query)
        data = None
        if body is not None:
            data = body if isinstance(body, bytes) else json.dumps(body).encode()
        req = urllib.request.Request(url, data=data, method=method)
        req.add_header("Accept", "application/json")
        if data is not None:
            req.add_header("Content-Type", content_type)
        if self.token:
            req.add_header("Authorization", f"Bearer {self.token}")
        try:
            with urllib.request.urlopen(req, timeout=self.timeout, context=self._ctx) as r:
                raw = r.read()
        except urllib.error.HTTPError as e:
            raise ApiError(e.code, e.read().decode(errors="replace")) from None
        except urllib.error.URLError as e:
            raise ApiError(0, str(e.reason)) from None
        return json.loads(raw) if raw else {}

    # ---- nodes -----------------------------------------------------------------------
    def get_node(self, name: str) -> dict:
        return self.request("GET", f"/api/v1/nodes/{name}")

    def list_nodes(self, label_selector: str | None = None) -> list[dict]:
        q = {"labelSelector": label_selector} if label_selector else None
        return self.request("GET", "/api/v1/nodes", query=q).get("items", [])

    def update_node(self, node: dict) -> dict:
        return self.request("PUT", f"/api/v1/nodes/{node['metadata']['name']}", node)

    def patch_node_annotations(self, name: str, annos: dict) -> dict:
        return self.request("PATCH", f"/api/v1/nodes/{name}",
                            {"metadata": {"annotations": annos}},
                            content_type="application/merge-patch+json")

    def patch_node_status(self, name: str, status: dict) -> dict:
        return self.request("PATCH", f"/api/v1/nodes/{name}/status", {"status": status},
                            content_type="application/merge-patch+json")

    # ---- pods ------------------------------------------------------------------------
    def get_pod(self, ns: str, name: str) -> dict:
        return self.request("GET", f"/api/v1/namespaces/{ns}/pods/{name}")

    def list_pods(self, namespace: str | None = None, field_selector: str | None = None,
                  label_selector: str | None = None) -> list[dict]:
        q = {}
        if field_selector:
            q["fieldSelector"] = field_selector
        if label_selector:
            q["labelSelector"] = label_selector
        path = f"/api/v1/namespaces/{namespace}/pods" if namespace else "/api/v1/pods"
        return self.request("GET", path, query=q or None).get("items", [])

    def list_pods_rv(self, field_selector: str | None = None) -> tuple[list[dict], str]:
        """LIST all pods; returns (items, list resourceVersion) to start a watch from."""
        q = {"fieldSelector": field_selector} if field_selector else None
        r = self.request("GET", "/api/v1/pods", query=q)
        return r.get("items", []), (r.get("metadata") or {}).get("resourceVersion", "0")

    def watch_pods(self, resource_version: str, timeout_s: float = 60.0,
                   field_selector: str | None = None):
        """WATCH pods from `resource_version`: yields (type, object) for ADDED /
        MODIFIED / DELETED / BOOKMARK events until the server ends the stream.
        An ERROR event (e.g. 410 Gone: the version was compacted) raises
        ApiError with its code; the caller relists."""
        q = {"watch": "1", "resourceVersion": resource_version, "allowWatchBookmarks": "true",
             "timeoutSeconds": str(int(timeout_s))}
        if field_selector:
            q["fieldSelector"] = field_selector
        url = self.server + "/api/v1/pods?" + urllib.parse.urlencode(q)
        req = urllib.request.Request(url, method="GET")
        req.add_header("Accept", "application/json")
        if self.token:
            req.add_header("Authorization", f"Bearer {self.token}")
        try:
            resp = urllib.request.urlopen(req, timeout=timeout_s + 10, context=self._ctx)
        except urllib.error.HTTPError as e:
            raise ApiError(e.code, e.read().decode(errors="replace")) from None
        except urllib.error.URLError as e:
            raise ApiError(0, str(e.reason)) from None
        with resp:
            for line in resp:
                line = line.strip()
                if not line:
                    continue
                ev = json.loads(line)
                if ev.get("type") == "ERROR":
                    st = ev.get("object") or {}
                    raise ApiError(int(st.get("code") or 500), st.get("message", ""))
                yield ev.get("type"), ev.get("object") or {}

    def patch_pod_annotations(self, ns: str, name: str, annos: dict) -> dict:
        return self.request("PATCH", f"/api/v1/namespaces/{ns}/pods/{name}",
                            {"metadata": {"annotations": annos}},
                            content_type="application/merge-patch+json")

    def bind_pod(self, ns: str, name: str, uid: str, node: str) -> dict:
        body = {"apiVersion": "v1", "kind": "Binding",
                "metadata": {"name": name, "namespace": ns, "uid": uid},
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        return self.request("POST", f"/api/v1/namespaces/{ns}/pods/{name}/binding", body)

    def create_pod(self, ns: str, pod: dict) -> dict:
        return self.request("POST", f"/api/v1/namespaces/{ns}/pods", pod)

    def delete_pod(self, ns: str, name: str) -> dict:
        return self.request("DELETE", f"/api/v1/namespaces/{ns}/pods/{name}")

    def create_node(self, node: dict) -> dict:
        return self.request("POST", "/api/v1/nodes", node)
