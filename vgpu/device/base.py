"""Vendor device abstraction and registry.

Reference: pkg/device/devices.go:20-25 (the `Devices` interface:
MutateAdmission, CheckType, GenerateResourceRequests, ParseConfig), :27-34
(`KnownDevice` handshake→register annotation map), :43-52 (registry init),
:54-91 (PodAllocationTrySuccess / Success / Failed), :93-101 (GlobalFlagSet).

The MI355X build registers one real vendor (`amd`) and, for tests and the
plumbing config (BASELINE.json config 1), a `fake` vendor with the same shape.
"""
from __future__ import annotations

import argparse
from abc import ABC, abstractmethod

from vgpu.api.resources import ContainerDeviceRequest, DeviceUsage


class Devices(ABC):
    """One accelerator vendor's admission/scheduling policy."""

    #: vendor type string carried in ContainerDeviceRequest.type / ContainerDevice.type
    vendor: str = ""
    #: node annotation keys (handshake, register)
    handshake_annotation: str = ""
    register_annotation: str = ""

    @abstractmethod
    def mutate_admission(self, ctr: dict) -> bool:
        """Mutate one container spec in place; True when it requests this vendor."""

    @abstractmethod
    def check_type(self, annos: dict, dev: DeviceUsage, req: ContainerDeviceRequest) -> tuple[bool, bool, bool]:
        """(found, pass, numa_assert) — found: this vendor owns the request type."""

    @abstractmethod
    def generate_resource_requests(self, ctr: dict) -> ContainerDeviceRequest:
        """Container spec → request (nums == 0 when the container asks for nothing)."""

    def parse_config(self, ap: argparse.ArgumentParser) -> None:
        """Register vendor flags."""

    def apply_config(self, ns: argparse.Namespace) -> None:
        """Consume parsed flags."""


_DEVICES: dict[str, Devices] = {}


def register(dev: Devices) -> None:
    _DEVICES[dev.vendor] = dev


def get_devices() -> dict[str, Devices]:
    if not _DEVICES:
        init_default_devices()
    return _DEVICES


def known_devices() -> dict[str, str]:
    """handshake annotation → register annotation."""
    return {d.handshake_annotation: d.register_annotation for d in get_devices().values()}


def init_default_devices(fake: bool = False) -> None:
    from .amd import AMDDevices
    _DEVICES.clear()
    register(AMDDevices())
    if fake:
        from .fake import FakeDevices
        register(FakeDevices())


def reset() -> None:
    _DEVICES.clear()


def resource_reqs(pod: dict) -> list[list[ContainerDeviceRequest]]:
    """Per container, per vendor requests (reference pkg/k8sutil/pod.go:26-40)."""
    from vgpu.k8s.objects import containers
    out = []
    for ctr in containers(pod):
        reqs = []
        for dev in get_devices().values():
            r = dev.generate_resource_requests(ctr)
            if r.nums > 0:
                reqs.append(r)
        out.append(reqs)
    return out
