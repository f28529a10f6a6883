"""In-process fake kube-apiserver for CPU-only end-to-end tests (the reference
has no fake API server at all — SURVEY.md §4: "no
k8s.io/client-go/kubernetes/fake, no kind/e2e").

Supports exactly the surface the stack uses: nodes GET/LIST/PUT/PATCH(+status)
/POST, pods GET/LIST (fieldSelector spec.nodeName=, labelSelector k=v)/POST/
PATCH/DELETE/binding, pod WATCH (`?watch=1&resourceVersion=N`: chunked
ADDED/MODIFIED/DELETED/BOOKMARK events, 410 Gone once N has been compacted),
JSON merge-patch (RFC 7386), resourceVersion conflicts (409) on PUT, and fault
injection (`inject`) for failure-path tests.
"""
from __future__ import annotations

import copy
import json
import re
import threading
import time
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse


def merge_patch(target, patch):
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


class FakeApiServer:
    def __init__(self):
        self.nodes: dict[str, dict] = {}
        self.pods: dict[tuple[str, str], dict] = {}
        self.rv = 0
        self.lock = threading.RLock()
        self.cond = threading.Condition(self.lock)
        self.events: list[tuple[int, str, dict]] = []  # pod watch history (rv, type, object)
        self.max_events = 2000
        self.events_floor = 0  # watches from a resourceVersion below this get 410 Gone
        self.faults: list[dict] = []
        self.requests: list[tuple[str, str]] = []
        self._srv: ThreadingHTTPServer | None = None
        self._stopping = False
        self._thread: threading.Thread | None = None

    # ---- store -----------------------------------------------------------------------
    def _bump(self, obj: dict) -> dict:
        self.rv += 1
        obj.setdefault("metadata", {})["resourceVersion"] = str(self.rv)
        return obj

    def add_node(self, name: str, annotations: dict | None = None, labels: dict | None = None) -> dict:
        with self.lock:
            n = {"apiVersion": "v1", "kind": "Node",
                 "metadata": {"name": name, "uid": str(uuid.uuid4()),
                              "annotations": dict(annotations or {}), "labels": dict(labels or {})},
                 "status": {"capacity": {}, "allocatable": {}}}
            self.nodes[name] = self._bump(n)
            return copy.deepcopy(n)

    def _event(self, typ: str, pod: dict) -> None:
        """Record a pod watch event (caller holds the lock) and wake watchers."""
        self.events.append((int(pod["metadata"]["resourceVersion"]), typ, copy.deepcopy(pod)))
        if len(self.events) > self.max_events:
            drop = len(self.events) - self.max_events
            self.events_floor = self.events[drop - 1][0]
            del self.events[:drop]
        self.cond.notify_all()

    def add_pod(self, pod: dict) -> dict:
        with self.lock:
            p = copy.deepcopy(pod)
            md = p.setdefault("metadata", {})
            md.setdefault("namespace", "default")
            md.setdefault("uid", str(uuid.uuid4()))
            md.setdefault("annotations", {})
            p.setdefault("spec", {})
            p.setdefault("status", {"phase": "Pending"})
            self.pods[(md["namespace"], md["name"])] = self._bump(p)
            self._event("ADDED", p)
            return copy.deepcopy(p)

    def delete_pod(self, ns: str, name: str) -> None:
        with self.lock:
            p = self.pods.pop((ns, name))
            self._event("DELETED", self._bump(p))

    def compact(self) -> None:
        """Drop the watch history (a watcher resuming from an old
        resourceVersion now gets 410 Gone and must relist)."""
        with self.lock:
            self.events.clear()
            self.rv += 1
            self.events_floor = self.rv

    def inject(self, method: str, path_regex: str, status: int, count: int = 1) -> None:
        with self.lock:
            self.faults.append({"method": method, "re": re.compile(path_regex), "status": status,
                                "count": count})

    def _fault(self, method: str, path: str) -> int | None:
        with self.lock:
            for f in self.faults:
                if f["count"] > 0 and f["method"] in (method, "*") and f["re"].search(path):
                    f["count"] -= 1
                    return f["status"]
        return None

    # ---- HTTP -----------------------------------------------------------------------
    def start(self, port: int = 0) -> str:
        server = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _send(self, code: int, obj) -> None:
                raw = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(raw)))
                self.end_headers()
                self.wfile.write(raw)

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n)) if n else None

            def _chunk(self, obj) -> None:
                raw = (json.dumps(obj) + "\n").encode()
                self.wfile.write(b"%x\r\n%s\r\n" % (len(raw), raw))
                self.wfile.flush()

            def _watch(self, q: dict) -> None:
                rv = int((q.get("resourceVersion") or ["0"])[0] or 0)
                timeout = float((q.get("timeoutSeconds") or ["30"])[0])
                bookmarks = (q.get("allowWatchBookmarks") or ["false"])[0] in ("true", "1")
                fs = (q.get("fieldSelector") or [""])[0]
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()
                deadline = time.monotonic() + timeout
                last_bookmark = time.monotonic()
                try:
                    while True:
                        with server.cond:
                            if rv < server.events_floor:
                                self._chunk({"type": "ERROR", "object": {
                                    "kind": "Status", "code": 410, "reason": "Expired",
                                    "message": f"too old resource version: {rv}"}})
                                break
                            batch = [e for e in server.events if e[0] > rv]
                            if not batch:
                                left = deadline - time.monotonic()
                                if left <= 0:
                                    break
                                server.cond.wait(min(left, 0.5))
                                batch = [e for e in server.events if e[0] > rv]
                            cur_rv = server.rv
                        for erv, typ, obj in batch:
                            rv = erv
                            if server._match_pod(obj, fs, ""):
                                self._chunk({"type": typ, "object": obj})
                        if bookmarks and time.monotonic() - last_bookmark > 1.0:
                            rv = max(rv, cur_rv)
                            self._chunk({"type": "BOOKMARK", "object": {
                                "kind": "Pod", "metadata": {"resourceVersion": str(rv)}}})
                            last_bookmark = time.monotonic()
                        if time.monotonic() >= deadline or server._stopping:
                            break
                    self.wfile.write(b"0\r\n\r\n")
                except (BrokenPipeError, ConnectionResetError):
                    pass

            def _handle(self, method: str):
                u = urlparse(self.path)
                server.requests.append((method, u.path))
                st = server._fault(method, u.path)
                if st:
                    self._body()
                    return self._send(st, {"kind": "Status", "code": st, "message": "injected"})
                q = parse_qs(u.query)
                if method == "GET" and (q.get("watch") or ["0"])[0] in ("1", "true") and u.path.endswith("/pods"):
                    return self._watch(q)
                try:
                    code, obj = server.route(method, u.path, q, self._body())
                except KeyError as e:
                    code, obj = 404, {"kind": "Status", "code": 404, "message": f"not found: {e}"}
                self._send(code, obj)

            def do_GET(self):
                self._handle("GET")

            def do_POST(self):
                self._handle("POST")

            def do_PUT(self):
                self._handle("PUT")

            def do_PATCH(self):
                self._handle("PATCH")

            def do_DELETE(self):
                self._handle("DELETE")

        self._srv = ThreadingHTTPServer(("127.0.0.1", port), H)
        self._srv.daemon_threads = True
        self._thread = threading.Thread(target=self._srv.serve_forever, daemon=True)
        self._thread.start()
        return f"http://127.0.0.1:{self._srv.server_address[1]}"

    def stop(self) -> None:
        self._stopping = True
        with self.cond:
            self.cond.notify_all()
        if self._srv:
            self._srv.shutdown()
            self._srv.server_close()

    # ---- routing ---------------------------------------------------------------------
    def route(self, method: str, path: str, q: dict, body):
        parts = [p for p in path.split("/") if p]
        with self.lock:
            if parts[:2] != ["api", "v1"]:
                return 404, {}
            rest = parts[2:]
            if rest and rest[0] == "nodes":
                return self._nodes(method, rest[1:], body)
            if rest and rest[0] == "pods" and method == "GET":
                return 200, {"kind": "PodList", "metadata": {"resourceVersion": str(self.rv)},
                             "items": self._list_pods(None, q)}
            if len(rest) >= 3 and rest[0] == "namespaces" and rest[2] == "pods":
                return self._pods(method, rest[1], rest[3:], q, body)
        return 404, {}

    def _nodes(self, method, rest, body):
        if not rest:
            if method == "GET":
                return 200, {"kind": "NodeList", "items": [copy.deepcopy(n) for n in self.nodes.values()]}
            if method == "POST":
                n = copy.deepcopy(body)
                self.nodes[n["metadata"]["name"]] = self._bump(n)
                return 201, copy.deepcopy(n)
        name = rest[0]
        node = self.nodes[name]
        if method == "GET":
            return 200, copy.deepcopy(node)
        if method == "PUT":
            rv = (body.get("metadata") or {}).get("resourceVersion")
            if rv and rv != node["metadata"]["resourceVersion"]:
                return 409, {"kind": "Status", "code": 409, "reason": "Conflict"}
            self.nodes[name] = self._bump(copy.deepcopy(body))
            return 200, copy.deepcopy(self.nodes[name])
        if method == "PATCH":
            self.nodes[name] = self._bump(merge_patch(node, body))
            return 200, copy.deepcopy(self.nodes[name])
        return 405, {}

    @staticmethod
    def _match_pod(p: dict, fs: str, ls: str) -> bool:
        for cond in filter(None, fs.split(",")):
            k, v = cond.split("=", 1)
            if k == "spec.nodeName" and (p.get("spec") or {}).get("nodeName", "") != v:
                return False
            if k == "status.phase" and (p.get("status") or {}).get("phase") != v:
                return False
        for cond in filter(None, ls.split(",")):
            k, v = cond.split("=", 1)
            if (p["metadata"].get("labels") or {}).get(k) != v:
                return False
        return True

    def _list_pods(self, ns, q):
        fs = (q.get("fieldSelector") or [""])[0]
        ls = (q.get("labelSelector") or [""])[0]
        return [copy.deepcopy(p) for (pns, _), p in self.pods.items()
                if (not ns or pns == ns) and self._match_pod(p, fs, ls)]

    def _pods(self, method, ns, rest, q, body):
        if not rest:
            if method == "GET":
                return 200, {"kind": "PodList", "metadata": {"resourceVersion": str(self.rv)},
                             "items": self._list_pods(ns, q)}
            if method == "POST":
                body.setdefault("metadata", {})["namespace"] = ns
                return 201, self.add_pod(body)
        name = rest[0]
        key = (ns, name)
        pod = self.pods[key]
        if len(rest) == 2 and rest[1] == "binding" and method == "POST":
            if (pod.get("spec") or {}).get("nodeName"):
                return 409, {"kind": "Status", "code": 409, "message": "already bound"}
            target = body["target"]["name"]
            if target not in self.nodes:
                return 404, {"kind": "Status", "code": 404, "message": "node not found"}
            pod["spec"]["nodeName"] = target
            self._bump(pod)
            self._event("MODIFIED", pod)
            return 201, {"kind": "Status", "status": "Success"}
        if method == "GET":
            return 200, copy.deepcopy(pod)
        if method == "PATCH":
            self.pods[key] = self._bump(merge_patch(pod, body))
            self._event("MODIFIED", self.pods[key])
            return 200, copy.deepcopy(self.pods[key])
        if method == "DELETE":
            self.delete_pod(ns, name)
            return 200, {"kind": "Status", "status": "Success"}
        return 405, {}
