"""Annotation codec round-trips (ports of the reference's
pkg/util/util_test.go:26-56 plus wire-format pins)."""
import pytest

from vgpu.api.codec import (CodecError, apply_node_devices_ext, decode_container_devices,
                            decode_node_devices, decode_pod_devices, encode_container_devices,
                            encode_node_devices, encode_node_devices_ext, encode_pod_devices)
from vgpu.api.resources import ContainerDevice, DeviceInfo


def test_empty_container_devices_coding():
    s = encode_container_devices([])
    assert decode_container_devices(s) == []


def test_empty_pod_device_coding():
    s = encode_pod_devices([])
    assert decode_pod_devices(s) == []


def test_pod_devices_coding():
    pd = [[ContainerDevice("UUID1", "Type1", 1000, 30)], [], [ContainerDevice("UUID1", "Type1", 1000, 30)]]
    s = encode_pod_devices(pd)
    assert s == "UUID1,Type1,1000,30:;;UUID1,Type1,1000,30:"
    assert decode_pod_devices(s) == pd


def test_node_devices_wire_format():
    devs = [DeviceInfo("GPU-0", 10, 294912, 100, "AMD-MI355X", 0, True),
            DeviceInfo("GPU-1", 10, 294912, 100, "AMD-MI355X", 1, False)]
    s = encode_node_devices(devs)
    assert s == "GPU-0,10,294912,100,AMD-MI355X,0,true:GPU-1,10,294912,100,AMD-MI355X,1,false:"
    back = decode_node_devices(s)
    assert [(d.id, d.count, d.devmem, d.devcore, d.type, d.numa, d.health) for d in back] == \
        [(d.id, d.count, d.devmem, d.devcore, d.type, d.numa, d.health) for d in devs]


def test_node_devices_reference_string():
    # a string as the reference's NVIDIA plugin writes it (register.go:102-120)
    s = "GPU-abc,10,32768,100,NVIDIA-Tesla V100-PCIE-32GB,0,true:"
    d = decode_node_devices(s)[0]
    assert d.type == "NVIDIA-Tesla V100-PCIE-32GB" and d.devmem == 32768 and d.health


def test_node_devices_bad():
    with pytest.raises(CodecError):
        decode_node_devices("no-colon-here")
    with pytest.raises(CodecError):
        decode_node_devices("a,b,c:")


def test_container_devices_missing_fields():
    with pytest.raises(CodecError):
        decode_container_devices("uuid,type:")
    assert decode_pod_devices("uuid,type:") == []


def test_ext_annotation_roundtrip():
    devs = [DeviceInfo("GPU-0", 4, 100, 100, "AMD-MI355X", cus=256, xgmi_hive="h1", index=3)]
    s = encode_node_devices_ext(devs)
    plain = decode_node_devices(encode_node_devices(devs))
    apply_node_devices_ext(plain, s)
    assert plain[0].cus == 256 and plain[0].xgmi_hive == "h1" and plain[0].index == 3
