"""Torch-free process group of the multi-GPU launch.

The rank processes of a partitioned run never import torch: torch ships its own ROCm runtime
(libamdhip64, libhsa-runtime64, rocBLAS, rocSOLVER, RCCL with the same SONAMEs as /opt/rocm), and
a process that imported it first would bind libaa_admm.so to that build instead of the one it
was compiled against (capi.check_runtime). torch.distributed.run stays the LAUNCHER only: it
exports RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR and MASTER_PORT, and this module does
the rest over plain sockets -- the RCCL unique-id broadcast, barriers, the max/sum of the bench
timings and the host transport's all-reduce.

Topology: a star around rank 0. A collective is: every other rank sends one frame to rank 0, rank
0 combines the frames in RANK ORDER and sends the result back, so every rank receives the same
bits (deterministic sums, no broadcast needed afterwards). Each frame carries an op tag; ranks
that disagree about which collective comes next fail loudly instead of mixing payloads.

Address: MASTER_PORT is held by the launcher's own store, so the group listens beside it. All
ranks on one node (LOCAL_WORLD_SIZE == WORLD_SIZE, the only launch bench.py makes): an abstract
Unix socket named after MASTER_ADDR:MASTER_PORT and the run id (unique while the launcher holds
the port). Otherwise TCP on MASTER_ADDR:MASTER_PORT+1 (AA_RDZV_PORT overrides the port).
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time

import numpy as np

_HDR = struct.Struct("<4sQ")   # op tag, payload bytes


class GroupError(RuntimeError):
    pass


class Group:
    def __init__(self, rank: int, size: int, address, family, timeout: float = 600.0):
        if not (0 <= rank < size):
            raise GroupError(f"bad rank {rank} of {size}")
        self.rank, self.size = rank, size
        self._peers = {}      # rank 0: {rank: socket}
        self._hub = None      # other ranks: socket to rank 0
        self._listener = None
        if size == 1:
            return
        deadline = time.time() + timeout
        if rank == 0:
            ls = socket.socket(family, socket.SOCK_STREAM)
            if family == socket.AF_INET:
                ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            ls.bind(address)
            ls.listen(size)
            ls.settimeout(max(1.0, deadline - time.time()))
            self._listener = ls
            while len(self._peers) < size - 1:
                try:
                    s, _ = ls.accept()
                except socket.timeout:
                    raise GroupError(f"rendezvous: {len(self._peers) + 1} of {size} ranks arrived "
                                     f"within {timeout:.0f} s") from None
                s.settimeout(None)
                self._nodelay(s, family)
                (r,) = struct.unpack("<i", self._recv_exact(s, 4))
                if not (0 < r < size) or r in self._peers:
                    raise GroupError(f"rendezvous: unexpected rank {r}")
                self._peers[r] = s
        else:
            while True:
                s = socket.socket(family, socket.SOCK_STREAM)
                try:
                    s.connect(address)
                    break
                except OSError:
                    s.close()
                    if time.time() > deadline:
                        raise GroupError(f"rendezvous: rank 0 not reachable within {timeout:.0f} s") from None
                    time.sleep(0.05)
            self._nodelay(s, family)
            s.sendall(struct.pack("<i", rank))
            self._hub = s

    # ---- construction -----------------------------------------------------------------
    @classmethod
    def from_env(cls, timeout: float = 600.0) -> "Group":
        """The group of a torch.distributed.run launch (or a single process when WORLD_SIZE is unset)."""
        size = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        if size == 1:
            return cls(0, 1, None, None)
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ["MASTER_PORT"])
        local = int(os.environ.get("LOCAL_WORLD_SIZE", str(size)))
        mode = os.environ.get("AA_RDZV", "unix" if local == size else "tcp")
        if mode == "unix":
            run_id = os.environ.get("TORCHELASTIC_RUN_ID", "")
            name = f"\0aa-admm.rdzv.{addr}:{port}.{run_id}"
            return cls(rank, size, name, socket.AF_UNIX, timeout)
        tport = int(os.environ.get("AA_RDZV_PORT", str(port + 1)))
        return cls(rank, size, (addr, tport), socket.AF_INET, timeout)

    # ---- collectives --------------------------------------------------------------------
    def barrier(self):
        self._collective(b"BARR", b"", lambda frames: b"")

    def broadcast_bytes(self, data: bytes | None, src: int = 0) -> bytes:
        """`data` from rank `src` to every rank."""
        mine = data if self.rank == src else b""
        if self.rank == src and data is None:
            raise GroupError("broadcast_bytes: the source rank passes the data")
        return self._collective(b"BCST", mine, lambda frames: frames[src])

    def allreduce_array(self, a: np.ndarray, op: str = "sum") -> np.ndarray:
        """In-place reduction of a contiguous float64 array; rank-order sum (or max/min) at rank 0,
        the same result bits on every rank."""
        if a.dtype != np.float64 or not a.flags.c_contiguous:
            raise GroupError("allreduce_array: contiguous float64 only")
        fn = {"sum": np.add, "max": np.maximum, "min": np.minimum}[op]

        def combine(frames):
            acc = np.frombuffer(frames[0], np.float64).copy()
            for f in frames[1:]:
                x = np.frombuffer(f, np.float64)
                if x.size != acc.size:
                    raise GroupError(f"allreduce_array: ranks disagree on the length ({x.size} vs {acc.size})")
                fn(acc, x, out=acc)
            return acc.tobytes()

        out = self._collective(b"ARED" if op == "sum" else b"AMAX" if op == "max" else b"AMIN", a.tobytes(), combine)
        a[...] = np.frombuffer(out, np.float64).reshape(a.shape)
        return a

    def allreduce_scalar(self, v: float, op: str = "sum") -> float:
        return float(self.allreduce_array(np.array([float(v)]), op)[0])

    def all_gather_json(self, obj) -> list:
        """Every rank's JSON-serialisable `obj`, in rank order, on every rank."""
        out = self._collective(b"AGTH", json.dumps(obj).encode(),
                               lambda frames: json.dumps([json.loads(f) for f in frames]).encode())
        return json.loads(out)

    def close(self):
        for s in list(self._peers.values()) + [self._hub, self._listener]:
            if s is not None:
                try:
                    s.close()
                except OSError:
                    pass
        self._peers, self._hub, self._listener = {}, None, None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- transport ----------------------------------------------------------------------
    @staticmethod
    def _nodelay(s, family):
        if family == socket.AF_INET:
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    @staticmethod
    def _recv_exact(s, n):
        buf = bytearray(n)
        view = memoryview(buf)
        got = 0
        while got < n:
            k = s.recv_into(view[got:], n - got)
            if k == 0:
                raise GroupError("rendezvous: a rank closed its connection")
            got += k
        return bytes(buf)

    def _send(self, s, tag, payload):
        s.sendall(_HDR.pack(tag, len(payload)))
        if payload:
            s.sendall(payload)

    def _recv(self, s, tag):
        t, n = _HDR.unpack(self._recv_exact(s, _HDR.size))
        if t != tag:
            raise GroupError(f"collective mismatch: expected {tag!r}, a rank sent {t!r}")
        return self._recv_exact(s, n) if n else b""

    def _collective(self, tag, payload, combine):
        if self.size == 1:
            return combine([payload])
        if self.rank != 0:
            self._send(self._hub, tag, payload)
            return self._recv(self._hub, tag)
        frames = [payload] + [self._recv(self._peers[r], tag) for r in range(1, self.size)]
        out = combine(frames)
        for r in range(1, self.size):
            self._send(self._peers[r], tag, out)
        return out
