"""Python wrappers of the native TCP key-value store (csrc/runtime/kv_store.cc)."""
from __future__ import annotations

import ctypes
import json
import struct

from .. import _native
from .._runtime_sigs import err


class KVServer:
    def __init__(self, host="0.0.0.0", port=0):
        self.lib = _native.runtime()
        bound = ctypes.c_int(0)
        self.h = self.lib.dtfrt_kv_server_start(host.encode(), int(port), ctypes.addressof(bound))
        if not self.h:
            raise OSError(err(self.lib))
        self.port = bound.value

    def stop(self):
        if self.h:
            self.lib.dtfrt_kv_server_stop(self.h)
            self.h = None


class KVClient:
    def __init__(self, host, port, timeout_s=300.0):
        self.lib = _native.runtime()
        self.h = self.lib.dtfrt_kv_connect(host.encode(), int(port), int(timeout_s * 1000))
        if not self.h:
            raise ConnectionError(err(self.lib))
        self.addr = (host, port)

    def set(self, key, value):
        b = value if isinstance(value, bytes) else (value.encode() if isinstance(value, str) else
                                                    json.dumps(value).encode())
        if self.lib.dtfrt_kv_set(self.h, key.encode(), b, len(b)):
            raise ConnectionError(err(self.lib))

    def get(self, key, timeout_s=None):
        """Blocking get: bytes, or None on timeout."""
        n = ctypes.c_uint64()
        st = self.lib.dtfrt_kv_get(self.h, key.encode(), -1 if timeout_s is None else int(timeout_s * 1000),
                                   ctypes.addressof(n))
        if st < 0:
            raise ConnectionError(err(self.lib))
        if st == 1:
            return None
        return ctypes.string_at(self.lib.dtfrt_kv_result(self.h), n.value)

    def get_json(self, key, timeout_s=None):
        b = self.get(key, timeout_s)
        return None if b is None else json.loads(b.decode())

    def add(self, key, delta=1):
        v = self.lib.dtfrt_kv_add(self.h, key.encode(), int(delta))
        if v == -(1 << 63):
            raise ConnectionError(err(self.lib))
        return v

    def counter(self, key):
        return self.add(key, 0)

    def check(self, key):
        return self.lib.dtfrt_kv_check(self.h, key.encode()) == 0

    def delete(self, key):
        self.lib.dtfrt_kv_del(self.h, key.encode())

    def wait_ge(self, key, target, timeout_s=None):
        cur = ctypes.c_int64()
        st = self.lib.dtfrt_kv_wait_ge(self.h, key.encode(), int(target), -1 if timeout_s is None else
                                       int(timeout_s * 1000), ctypes.addressof(cur))
        if st < 0:
            raise ConnectionError(err(self.lib))
        return st == 0

    def keys(self, prefix=""):
        n = ctypes.c_uint64()
        self.lib.dtfrt_kv_keys(self.h, prefix.encode(), ctypes.addressof(n))
        s = ctypes.string_at(self.lib.dtfrt_kv_result(self.h), n.value).decode()
        return [k for k in s.split("\n") if k]

    def barrier(self, name, n, timeout_s=None):
        self.add(f"barrier/{name}", 1)
        return self.wait_ge(f"barrier/{name}", n, timeout_s)

    def close(self):
        if self.h:
            self.lib.dtfrt_kv_close(self.h)
            self.h = None


def pack_i64(v):
    return struct.pack("<q", int(v))


def unpack_i64(b):
    return struct.unpack("<q", b)[0]
