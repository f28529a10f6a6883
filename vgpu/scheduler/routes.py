"""HTTP(S) routes of the extender: POST /filter (ExtenderArgs →
ExtenderFilterResult), POST /bind (ExtenderBindingArgs → ExtenderBindingResult),
POST /webhook (AdmissionReview), GET /healthz, GET /nodes (debug view of the
registry and usage).

Reference: pkg/scheduler/routes/route.go:41-80 (PredicateRoute), :82-111 (Bind),
:125-134 (WebHookRoute); cmd/scheduler/main.go:73-76.
"""
from __future__ import annotations

import json
import logging
import ssl
import threading
from dataclasses import asdict
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .webhook import handle_admission

log = logging.getLogger("vgpu.scheduler.routes")


def make_handler(scheduler):
    class Handler(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, fmt, *a):
            log.debug(fmt, *a)

        def _reply(self, code: int, obj) -> None:
            raw = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(raw)))
            self.end_headers()
            self.wfile.write(raw)

        def _json(self):
            n = int(self.headers.get("Content-Length") or 0)
            raw = self.rfile.read(n) if n else b""
            return json.loads(raw) if raw else {}

        def do_GET(self):
            if self.path == "/healthz":
                return self._reply(200, {"status": "ok"})
            if self.path == "/nodes":
                usage, _ = scheduler.nodes_usage(None)
                return self._reply(200, {k: [asdict(d) for d in v.devices] for k, v in usage.items()})
            self._reply(404, {"error": "not found"})

        def do_POST(self):
            try:
                body = self._json()
            except ValueError as e:
                return self._reply(400, {"error": f"bad json: {e}"})
            try:
                if self.path == "/filter":
                    return self._reply(200, scheduler.filter(body))
                if self.path == "/bind":
                    return self._reply(200, scheduler.bind(body))
                if self.path == "/webhook":
                    return self._reply(200, handle_admission(body))
            except Exception as e:  # never crash the server on one request
                log.exception("handler error")
                return self._reply(500, {"error": str(e)})
            self._reply(404, {"error": "not found"})

    return Handler


def serve(scheduler, bind: str, cert_file: str = "", key_file: str = "",
          background: bool = False) -> ThreadingHTTPServer:
    host, _, port = bind.rpartition(":")
    srv = ThreadingHTTPServer((host or "0.0.0.0", int(port)), make_handler(scheduler))
    srv.daemon_threads = True
    if cert_file and key_file:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(cert_file, key_file)
        srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
    if background:
        threading.Thread(target=srv.serve_forever, daemon=True, name="vgpu-extender").start()
    else:
        srv.serve_forever()
    return srv
