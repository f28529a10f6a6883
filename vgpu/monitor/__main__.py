"""Node monitor daemon: region discovery + GC, priority feedback every 5 s,
Prometheus metrics on :9394, JSON node view on /nodeinfo.

Reference: cmd/vGPUmonitor/main.go:11-32 (gRPC server + metrics + feedback
loop), feedback.go:257-269 (watchAndFeedback), metrics.go:262-293 (:9394);
the reference's NodeVGPUInfo gRPC service is declared but unimplemented
(pathmonitor.go:122-134), so it is replaced by a real JSON endpoint.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import threading
from dataclasses import asdict
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from prometheus_client import REGISTRY, start_http_server

from .feedback import observe
from .metrics import MonitorCollector
from .pathmonitor import PathMonitor
from .pids import resolve_and_purge

log = logging.getLogger("vgpu.monitor")


def node_info(pm: PathMonitor) -> dict:
    return {key: {"pod": cr.pod_name, "namespace": cr.namespace, "container": cr.ctr_name,
                  "priority": cr.region.priority, "recent_kernel": cr.region.recent_kernel,
                  "utilization_switch": cr.region.utilization_switch,
                  "devices": [asdict(d) | {"cu_mask": hex(d.cu_mask)} for d in cr.region.devices()]}
            for key, cr in pm.regions.items()}


def serve_nodeinfo(pm: PathMonitor, port: int, host: str = "0.0.0.0") -> ThreadingHTTPServer:
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            if self.path not in ("/nodeinfo", "/healthz"):
                self.send_response(404)
                self.end_headers()
                return
            raw = json.dumps(node_info(pm) if self.path == "/nodeinfo" else {"status": "ok"}).encode()
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(raw)))
            self.end_headers()
            self.wfile.write(raw)

    srv = ThreadingHTTPServer((host, port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="vgpu-monitor")
    ap.add_argument("--containers-dir", default=os.environ.get("VGPU_CONTAINERS_DIR",
                                                                "/usr/local/vgpu/containers"))
    ap.add_argument("--metrics-port", type=int, default=9394)
    ap.add_argument("--nodeinfo-port", type=int, default=9396)
    ap.add_argument("--interval", type=float, default=5.0)
    ap.add_argument("--backend", default=os.environ.get("VGPU_BACKEND", "auto"))
    ap.add_argument("--no-kube", action="store_true", help="run without API server access")
    ns = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    client = None
    if not ns.no_kube:
        from vgpu.k8s.client import KubeClient
        client = KubeClient.from_env()
    node = os.environ.get("NODE_NAME") or os.environ.get("NodeName", "")
    pm = PathMonitor(ns.containers_dir, client, node)
    backend = None
    try:
        from vgpu.deviceplugin.discovery import load_backend
        backend = load_backend(ns.backend)
    except Exception as e:
        log.warning("no device backend (%s); host metrics disabled", e)
    REGISTRY.register(MonitorCollector(pm, backend))
    start_http_server(ns.metrics_port)
    serve_nodeinfo(pm, ns.nodeinfo_port)
    stop = threading.Event()
    while not stop.wait(ns.interval):
        try:
            pm.scan()
            resolve_and_purge(pm.regions)  # host pids the shim could not verify; dead slots freed
            observe({k: cr.region for k, cr in pm.regions.items()})
        except Exception as e:
            log.error("monitor pass failed: %s", e)
    return 0


if __name__ == "__main__":
    sys.exit(main())
