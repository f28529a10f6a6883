"""A second, fake vendor with the same policy shape, for the CPU-only plumbing
configuration (BASELINE.json config 1) and multi-vendor scheduler tests."""
from __future__ import annotations

from vgpu.api.resources import ContainerDeviceRequest, DeviceUsage
from vgpu.k8s.objects import limit_or_request, parse_quantity

from .base import Devices

FAKE_VENDOR = "FAKE"


class FakeDevices(Devices):
    vendor = FAKE_VENDOR
    handshake_annotation = "4pd.io/node-handshake-fake"
    register_annotation = "4pd.io/node-fake-register"
    resource_count = "fake.com/vgpu"
    resource_mem = "fake.com/vgpumem"
    resource_cores = "fake.com/vgpucores"

    def mutate_admission(self, ctr: dict) -> bool:
        return limit_or_request(ctr, self.resource_count) is not None

    def check_type(self, annos: dict, dev: DeviceUsage, req: ContainerDeviceRequest):
        if req.type == self.vendor:
            return True, True, False
        return False, False, False

    def generate_resource_requests(self, ctr: dict) -> ContainerDeviceRequest:
        n = parse_quantity(limit_or_request(ctr, self.resource_count))
        if not n:
            return ContainerDeviceRequest(nums=0)
        mem = parse_quantity(limit_or_request(ctr, self.resource_mem)) or 0
        cores = parse_quantity(limit_or_request(ctr, self.resource_cores)) or 0
        return ContainerDeviceRequest(nums=n, type=self.vendor, memreq=mem,
                                      mem_percentage=101 if mem else 100, coresreq=cores)
