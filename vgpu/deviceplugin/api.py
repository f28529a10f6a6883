"""kubelet device-plugin API v1beta1, built at runtime (no protoc in this
environment): a FileDescriptorProto identical in wire format to
k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto, message classes from
it, and grpc generic handlers / client stubs for the `Registration` and
`DevicePlugin` services.

Reference: the Go plugin uses the generated pluginapi package
(pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:237-495).
"""
from __future__ import annotations

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

VERSION = "v1beta1"
KUBELET_SOCKET = "kubelet.sock"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

_T = descriptor_pb2.FieldDescriptorProto
_STR, _BOOL, _I64, _I32, _MSG = _T.TYPE_STRING, _T.TYPE_BOOL, _T.TYPE_INT64, _T.TYPE_INT32, _T.TYPE_MESSAGE
_OPT, _REP = _T.LABEL_OPTIONAL, _T.LABEL_REPEATED

# message name -> [(field, number, type, label, type_name)]
_MESSAGES = {
    "DevicePluginOptions": [("pre_start_required", 1, _BOOL, _OPT, None),
                            ("get_preferred_allocation_available", 2, _BOOL, _OPT, None)],
    "RegisterRequest": [("version", 1, _STR, _OPT, None), ("endpoint", 2, _STR, _OPT, None),
                        ("resource_name", 3, _STR, _OPT, None),
                        ("options", 4, _MSG, _OPT, "DevicePluginOptions")],
    "Empty": [],
    "ListAndWatchResponse": [("devices", 1, _MSG, _REP, "Device")],
    "TopologyInfo": [("nodes", 1, _MSG, _REP, "NUMANode")],
    "NUMANode": [("ID", 1, _I64, _OPT, None)],
    "Device": [("ID", 1, _STR, _OPT, None), ("health", 2, _STR, _OPT, None),
               ("topology", 3, _MSG, _OPT, "TopologyInfo")],
    "PreStartContainerRequest": [("devices_ids", 1, _STR, _REP, None)],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, _MSG, _REP, "ContainerPreferredAllocationRequest")],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, _STR, _REP, None),
                                            ("must_include_deviceIDs", 2, _STR, _REP, None),
                                            ("allocation_size", 3, _I32, _OPT, None)],
    "PreferredAllocationResponse": [("container_responses", 1, _MSG, _REP, "ContainerPreferredAllocationResponse")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, _STR, _REP, None)],
    "AllocateRequest": [("container_requests", 1, _MSG, _REP, "ContainerAllocateRequest")],
    "ContainerAllocateRequest": [("devices_ids", 1, _STR, _REP, None)],
    "CDIDevice": [("name", 1, _STR, _OPT, None)],
    "AllocateResponse": [("container_responses", 1, _MSG, _REP, "ContainerAllocateResponse")],
    "ContainerAllocateResponse": [("envs", 1, "map", _REP, None), ("mounts", 2, _MSG, _REP, "Mount"),
                                  ("devices", 3, _MSG, _REP, "DeviceSpec"),
                                  ("annotations", 4, "map", _REP, None),
                                  ("cdi_devices", 5, _MSG, _REP, "CDIDevice")],
    "Mount": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
              ("read_only", 3, _BOOL, _OPT, None)],
    "DeviceSpec": [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
                   ("permissions", 3, _STR, _OPT, None)],
}

_SERVICES = {
    "Registration": [("Register", "RegisterRequest", "Empty", False)],
    "DevicePlugin": [("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
                     ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
                     ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
                     ("Allocate", "AllocateRequest", "AllocateResponse", False),
                     ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False)],
}


def _camel(s: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in s.split("_"))


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="vgpu_deviceplugin_v1beta1.proto", package=VERSION,
                                            syntax="proto3")
    for mname, fields in _MESSAGES.items():
        m = fd.message_type.add(name=mname)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, label=label)
            if typ == "map":
                entry = m.nested_type.add(name=_camel(fname) + "Entry")
                entry.options.map_entry = True
                entry.field.add(name="key", number=1, type=_STR, label=_OPT)
                entry.field.add(name="value", number=2, type=_STR, label=_OPT)
                f.type = _MSG
                f.type_name = f".{VERSION}.{mname}.{entry.name}"
            else:
                f.type = typ
                if tname:
                    f.type_name = f".{VERSION}.{tname}"
    for sname, methods in _SERVICES.items():
        s = fd.service.add(name=sname)
        for meth, req, resp, stream in methods:
            s.method.add(name=meth, input_type=f".{VERSION}.{req}", output_type=f".{VERSION}.{resp}",
                         server_streaming=stream)
    pool = descriptor_pool.DescriptorPool()
    fdesc = pool.Add(fd)
    fdesc = pool.FindFileByName(fd.name)
    classes = {}
    for mname in _MESSAGES:
        classes[mname] = message_factory.GetMessageClass(fdesc.message_types_by_name[mname])
    return classes


M = _build()

DevicePluginOptions = M["DevicePluginOptions"]
RegisterRequest = M["RegisterRequest"]
Empty = M["Empty"]
ListAndWatchResponse = M["ListAndWatchResponse"]
TopologyInfo = M["TopologyInfo"]
NUMANode = M["NUMANode"]
Device = M["Device"]
PreStartContainerRequest = M["PreStartContainerRequest"]
PreStartContainerResponse = M["PreStartContainerResponse"]
PreferredAllocationRequest = M["PreferredAllocationRequest"]
PreferredAllocationResponse = M["PreferredAllocationResponse"]
ContainerPreferredAllocationResponse = M["ContainerPreferredAllocationResponse"]
AllocateRequest = M["AllocateRequest"]
AllocateResponse = M["AllocateResponse"]
ContainerAllocateRequest = M["ContainerAllocateRequest"]
ContainerAllocateResponse = M["ContainerAllocateResponse"]
Mount = M["Mount"]
DeviceSpec = M["DeviceSpec"]
CDIDevice = M["CDIDevice"]


def service_handler(service: str, impl) -> grpc.GenericRpcHandler:
    """Generic handler dispatching every method of `service` to impl.<Method>(request, context)."""
    handlers = {}
    for meth, req, resp, stream in _SERVICES[service]:
        fn = getattr(impl, meth)
        kw = dict(request_deserializer=M[req].FromString, response_serializer=M[resp].SerializeToString)
        handlers[meth] = (grpc.unary_stream_rpc_method_handler(fn, **kw) if stream
                          else grpc.unary_unary_rpc_method_handler(fn, **kw))
    return grpc.method_handlers_generic_handler(f"{VERSION}.{service}", handlers)


class Stub:
    """Client stub for either service over a channel."""

    def __init__(self, channel: grpc.Channel, service: str):
        for meth, req, resp, stream in _SERVICES[service]:
            path = f"/{VERSION}.{service}/{meth}"
            mk = channel.unary_stream if stream else channel.unary_unary
            setattr(self, meth, mk(path, request_serializer=M[req].SerializeToString,
                                   response_deserializer=M[resp].FromString))


def unix_target(path: str) -> str:
    return f"unix://{path}"
