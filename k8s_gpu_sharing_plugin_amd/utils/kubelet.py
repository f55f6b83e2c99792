"""An independent kubelet-side implementation on grpcio (gRPC C-core) + protobuf.

The daemon's gRPC/HTTP2 transport and protobuf codec are hand-written on
nghttp2; talking to them from grpcio -- the same C-core family kubelet's
grpc-go interoperates with -- checks wire compatibility with an implementation
that shares no code with ours. Message classes come from
proto/deviceplugin/v1beta1/api.proto via protoc's descriptor set.
"""

import queue
import threading
from concurrent import futures

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from .build import build_descriptor

_pool = None
_classes = {}


def messages():
    """Dict of v1beta1 message classes (RegisterRequest, AllocateRequest, ...)."""
    global _pool
    if not _classes:
        with open(build_descriptor(), "rb") as f:
            fds = descriptor_pb2.FileDescriptorSet.FromString(f.read())
        _pool = descriptor_pool.DescriptorPool()
        for fd in fds.file:
            _pool.Add(fd)
        fd = _pool.FindFileByName("deviceplugin/v1beta1/api.proto")
        for name in fd.message_types_by_name:
            _classes[name] = message_factory.GetMessageClass(fd.message_types_by_name[name])
    return _classes


class StubKubelet:
    """Serves v1beta1.Registration on `socket_path` and records registrations."""

    def __init__(self, socket_path: str, reject_with: str = ""):
        m = messages()
        self.socket_path = socket_path
        self.registrations = queue.Queue()
        self.reject_with = reject_with
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))

        def register(req, ctx):
            if self.reject_with:
                ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, self.reject_with)
            self.registrations.put(req)
            return m["Empty"]()

        handler = grpc.method_handlers_generic_handler("v1beta1.Registration", {
            "Register": grpc.unary_unary_rpc_method_handler(
                register, request_deserializer=m["RegisterRequest"].FromString,
                response_serializer=m["Empty"].SerializeToString),
        })
        self._server.add_generic_rpc_handlers((handler,))
        self._server.add_insecure_port("unix:" + socket_path)

    def start(self):
        self._server.start()
        return self

    def stop(self):
        # Wait for the shutdown to finish: grpcio removes the socket file when it
        # does, which would otherwise delete a new kubelet's socket at the same path.
        self._server.stop(0).wait(10)

    def wait_registration(self, timeout=10.0):
        return self.registrations.get(timeout=timeout)


class PluginClient:
    """kubelet -> plugin calls over the plugin's Unix socket."""

    def __init__(self, socket_path: str):
        m = messages()
        self.m = m
        # Own subchannel pool: every client is its own connection (grpcio would
        # otherwise share one between channels to the same target).
        self.channel = grpc.insecure_channel("unix:" + socket_path,
                                             options=[("grpc.use_local_subchannel_pool", 1)])
        svc = "/v1beta1.DevicePlugin/"

        def uu(name, req, resp):
            return self.channel.unary_unary(svc + name, request_serializer=m[req].SerializeToString,
                                            response_deserializer=m[resp].FromString)

        self._options = uu("GetDevicePluginOptions", "Empty", "DevicePluginOptions")
        self._allocate = uu("Allocate", "AllocateRequest", "AllocateResponse")
        self._preferred = uu("GetPreferredAllocation", "PreferredAllocationRequest",
                             "PreferredAllocationResponse")
        self._prestart = uu("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse")
        self._law = self.channel.unary_stream(svc + "ListAndWatch",
                                              request_serializer=m["Empty"].SerializeToString,
                                              response_deserializer=m["ListAndWatchResponse"].FromString)

    def close(self):
        self.channel.close()

    def options(self, timeout=5):
        return self._options(self.m["Empty"](), timeout=timeout)

    def allocate(self, *containers, timeout=5):
        req = self.m["AllocateRequest"]()
        for ids in containers:
            req.container_requests.add().devicesIDs.extend(ids)
        return self._allocate(req, timeout=timeout)

    def preferred(self, available, must_include=(), size=1, timeout=5):
        req = self.m["PreferredAllocationRequest"]()
        c = req.container_requests.add()
        c.available_deviceIDs.extend(available)
        c.must_include_deviceIDs.extend(must_include)
        c.allocation_size = size
        return self._preferred(req, timeout=timeout)

    def prestart(self, ids=(), timeout=5):
        req = self.m["PreStartContainerRequest"]()
        req.devicesIDs.extend(ids)
        return self._prestart(req, timeout=timeout)

    def watch(self):
        """Starts ListAndWatch in a thread; returns (queue of responses, call)."""
        call = self._law(self.m["Empty"]())
        q = queue.Queue()

        def pump():
            try:
                for resp in call:
                    q.put(resp)
            except grpc.RpcError as e:  # cancelled / server gone
                q.put(e)
            q.put(None)

        threading.Thread(target=pump, daemon=True).start()
        return q, call
