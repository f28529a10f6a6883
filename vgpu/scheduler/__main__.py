"""Scheduler extender + webhook daemon.

Reference: cmd/scheduler/main.go:48-61 (flags --http_bind, --cert_file,
--key_file, --scheduler-name, --default-mem, --default-cores, vendor
resource-name flags), :63-87 (start informer, registration loop, metrics on
:9395, routes).

    python -m vgpu.scheduler --http-bind 0.0.0.0:443 --cert-file ... --key-file ...
"""
from __future__ import annotations

import argparse
import logging
import sys

from prometheus_client import REGISTRY, start_http_server

from vgpu import config
from vgpu.config import SchedulerConfig, add_dataclass_args, from_namespace
from vgpu.device.base import get_devices, init_default_devices
from vgpu.k8s.client import KubeClient

from .core import Scheduler
from .metrics import SchedulerCollector
from .routes import serve


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="vgpu-scheduler")
    add_dataclass_args(ap, SchedulerConfig)
    ap.add_argument("--fake-vendor", action="store_true", help="also register the fake vendor")
    ap.add_argument("-v", "--verbose", action="count", default=0)
    init_default_devices()
    for d in get_devices().values():
        d.parse_config(ap)
    ns = ap.parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if ns.verbose else logging.INFO,
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    if ns.fake_vendor:
        init_default_devices(fake=True)
    for d in get_devices().values():
        d.apply_config(ns)
    cfg = from_namespace(SchedulerConfig, ns)
    config.SCHEDULER = cfg
    sched = Scheduler(KubeClient.from_env(), cfg)
    sched.resync_pods()
    sched.run_loops()
    REGISTRY.register(SchedulerCollector(sched))
    mhost, _, mport = cfg.metrics_bind.rpartition(":")
    start_http_server(int(mport), addr=mhost or "0.0.0.0")
    serve(sched, cfg.http_bind, cfg.cert_file, cfg.key_file)
    return 0


if __name__ == "__main__":
    sys.exit(main())
