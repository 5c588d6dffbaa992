"""Drives the erl_nif shim (emqx_amd/csrc/nif/emqx_tm_nif.c) through the test
stand-in for the Erlang runtime (tests/nif_mock, built into
emqx_amd/libemqx_nif_mock.so by emqx_amd.build).  Python values map to terms:
bytes -> binary, str -> atom, int -> integer, tuple -> tuple, list -> list,
Ref -> reference, Raw -> a term handle returned earlier (the engine)."""

from __future__ import annotations

import ast
import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("EMQX_NIF_MOCK_LIB") or os.path.join(HERE, "..", "emqx_amd", "libemqx_nif_mock.so")

TERM = C.c_size_t


class Raw:
    def __init__(self, handle):
        self.handle = handle


class Ref:
    def __init__(self, handle, ident):
        self.handle, self.ident = handle, ident


class Nif:
    _lock = threading.Lock()
    _lib = None

    def __init__(self):
        with Nif._lock:
            if Nif._lib is None:
                L = C.CDLL(LIB)
                for name, res, args in [
                    ("mock_atom", TERM, [C.c_char_p]), ("mock_int", TERM, [C.c_int64]),
                    ("mock_bin", TERM, [C.c_char_p, C.c_size_t]), ("mock_list", TERM, [C.c_void_p, C.c_uint]),
                    ("mock_tuple", TERM, [C.c_void_p, C.c_uint]), ("mock_ref", TERM, []),
                    ("mock_process", C.c_void_p, [C.c_int]), ("mock_load", C.c_int, []),
                    ("mock_nif_flags", C.c_int, [C.c_char_p, C.c_uint]),
                    ("mock_call", TERM, [C.c_char_p, C.c_uint, C.c_void_p, C.c_void_p]),
                    ("mock_recv", TERM, [C.c_int, C.c_int]),
                    ("mock_tuple_elem", TERM, [TERM, C.c_uint]),
                    ("mock_drop_resource_term", None, [TERM]), ("mock_live_resources", C.c_int, []),
                    ("mock_format", C.c_size_t, [TERM, C.c_char_p, C.c_size_t]),
                ]:
                    f = getattr(L, name)
                    f.restype, f.argtypes = res, args
                assert L.mock_load() == 0
                Nif._lib = L
        self.L = Nif._lib
        self._envs = {}

    # ---- terms ----
    def term(self, v) -> int:
        L = self.L
        if isinstance(v, Raw):
            return v.handle
        if isinstance(v, Ref):
            return v.handle
        if isinstance(v, (bytes, bytearray)):
            return L.mock_bin(bytes(v), len(v))
        if isinstance(v, str):
            return L.mock_atom(v.encode())
        if isinstance(v, bool):
            return L.mock_atom(b"true" if v else b"false")
        if isinstance(v, int):
            return L.mock_int(v)
        if isinstance(v, (tuple, list)):
            arr = (TERM * max(len(v), 1))(*[self.term(x) for x in v])
            return (L.mock_tuple if isinstance(v, tuple) else L.mock_list)(arr, len(v))
        raise TypeError(type(v))

    def ref(self) -> Ref:
        h = self.L.mock_ref()
        return Ref(h, self.decode(h)[1])

    def decode(self, t: int):
        n = self.L.mock_format(t, None, 0)
        buf = C.create_string_buffer(n)
        self.L.mock_format(t, buf, n)
        return ast.literal_eval(buf.value.decode())

    # ---- calls ----
    def env(self, pid: int):
        with Nif._lock:
            if pid not in self._envs:
                self._envs[pid] = self.L.mock_process(pid)
            return self._envs[pid]

    def call_raw(self, name: str, *args, pid: int = 1) -> int:
        arr = (TERM * max(len(args), 1))(*[self.term(a) for a in args])
        t = self.L.mock_call(name.encode(), len(args), self.env(pid), arr)
        assert t, f"no NIF {name}/{len(args)}"
        return t

    def call(self, name: str, *args, pid: int = 1):
        return self.decode(self.call_raw(name, *args, pid=pid))

    def flags(self, name: str, arity: int) -> int:
        return self.L.mock_nif_flags(name.encode(), arity)

    def recv(self, pid: int, timeout_ms: int = 10000):
        t = self.L.mock_recv(pid, timeout_ms)
        return None if not t else self.decode(t)

    def new(self, device: int) -> Raw:
        t = self.call_raw("new", device)
        ok = self.decode(t)
        assert ok[0] == "ok", ok
        return Raw(self.L.mock_tuple_elem(t, 1))

    def drop(self, engine: Raw):
        self.L.mock_drop_resource_term(engine.handle)

    def live_resources(self) -> int:
        return self.L.mock_live_resources()

    def match(self, engine: Raw, topic: bytes, pid: int = 1, timeout_ms: int = 30000):
        """emqx_tm:match/2 as the Erlang module does it: match_async + receive."""
        r = self.ref()
        rc = self.call("match_async", engine, topic, r, pid=pid)
        if rc != "ok":
            return rc
        msg = self.recv(pid, timeout_ms)
        assert msg is not None, "no reply"
        assert msg[0] == "emqx_tm_match" and msg[1] == ("#ref", r.ident), msg
        return msg[2]

