"""Single-writer / multi-reader broadcast of per-step inputs through POSIX shared
memory (the "shm broadcast for step metadata" of SURVEY.md §5 / §2.7).

Tensor-parallel rank 0 owns the scheduler; every decode step it must hand the
other ranks the same host inputs (token ids, positions, slot mapping, block
tables, sampling parameters) before they can enter the step's collectives.
Sending them through RCCL would cost a device round trip per step; a pickle
through a /dev/shm ring costs a few microseconds.

Layout (one file in /dev/shm, mmap'ed by every rank; no multiprocessing
resource tracker involved, the writer unlinks it on close / exit)::

    [0:8)                       write sequence number of the newest message
    [8:8+8*R)                   per-reader ack sequence numbers
    slot i (N slots, each S B): [seq u64][len u64][payload ...]

The writer waits until every reader has acked the message that previously
occupied a slot before overwriting it; a reader polls the next slot's ``seq``.
x86-64 stores are not reordered with other stores, so writing the payload
before the slot's ``seq`` publishes it safely.  Messages larger than a slot go
into a fresh overflow segment whose name is sent in the slot instead.
"""
from __future__ import annotations

import atexit
import mmap
import os
import pickle
import time
import uuid
from typing import Any, Optional

import numpy as np

_HDR = 16
_DIR = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"


class _Seg:
    """A named, mmap'ed shared-memory file."""

    def __init__(self, name: str, size: int = 0, create: bool = False):
        self.name = name
        self.path = os.path.join(_DIR, name)
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(self.path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, size)
            else:
                size = os.fstat(fd).st_size
            self.mm = mmap.mmap(fd, size)
        finally:
            os.close(fd)
        self.buf = memoryview(self.mm)
        self.size = size

    def close(self):
        try:
            self.buf.release()
            self.mm.close()
        except Exception:
            pass

    def unlink(self):
        try:
            os.unlink(self.path)
        except FileNotFoundError:
            pass


class PeerDied(RuntimeError):
    """The other side of the broadcast ring is gone (TP worker or rank 0 died)."""


class ShmBroadcast:
    def __init__(self, num_readers: int, name: Optional[str] = None, create: bool = True,
                 reader_index: int = -1, num_slots: int = 8, slot_bytes: int = 4 << 20):
        self.num_readers = num_readers
        self.num_slots = num_slots
        self.slot_bytes = slot_bytes
        self.reader_index = reader_index
        size = 8 + 8 * num_readers + num_slots * slot_bytes
        if create:
            self.name = name or f"ft_bcast_{os.getpid()}_{uuid.uuid4().hex[:8]}"
            self.shm = _Seg(self.name, size, create=True)
            atexit.register(self.close)
            self.shm.buf[: 8 + 8 * num_readers] = b"\0" * (8 + 8 * num_readers)
            for i in range(num_slots):
                off = self._slot_off(i)
                self.shm.buf[off:off + 8] = np.int64(-1).tobytes()
        else:
            self.name = name
            self.shm = _Seg(name)
        self.owner = create
        self.liveness = None  # optional () -> bool, polled while blocked (~1/s)
        self._hdr = np.ndarray((1 + num_readers,), dtype=np.int64, buffer=self.shm.buf, offset=0)
        self._seq = int(self._hdr[0])
        # messages are numbered from 1; a reader's ack is the last one it consumed
        self._next = int(self._hdr[1 + reader_index]) + 1 if reader_index >= 0 else 0

    # ------------------------------------------------------------------ helpers
    def _slot_off(self, i: int) -> int:
        return 8 + 8 * self.num_readers + i * self.slot_bytes

    def _slot_hdr(self, i: int) -> np.ndarray:
        return np.ndarray((2,), dtype=np.int64, buffer=self.shm.buf, offset=self._slot_off(i))

    def _spin(self, cond, timeout: Optional[float]):
        t0 = time.perf_counter()
        n = 0
        while not cond():
            n += 1
            if n > 200:
                time.sleep(5e-5 if n < 20000 else 1e-3)
                # a dead peer never acks / never sends: ask the owner's liveness
                # probe about once a second instead of spinning forever
                if n >= 20000 and n % 1000 == 0 and self.liveness is not None and not self.liveness():
                    raise PeerDied("shm broadcast peer process died")
            if timeout is not None and time.perf_counter() - t0 > timeout:
                raise TimeoutError("shm broadcast timed out")

    # ------------------------------------------------------------------ writer
    def send(self, obj: Any, timeout: Optional[float] = None):
        assert self.owner, "only the creating rank writes"
        data = pickle.dumps(obj, protocol=5)
        seq = self._seq + 1
        slot = seq % self.num_slots
        acks = self._hdr[1:]
        old = seq - self.num_slots  # message previously in this slot
        if old >= 1:
            self._spin(lambda: int(acks.min()) >= old, timeout)
        h = self._slot_hdr(slot)
        off = self._slot_off(slot) + _HDR
        if len(data) <= self.slot_bytes - _HDR:
            self.shm.buf[off:off + len(data)] = data
            h[1] = len(data)
        else:  # overflow: payload in its own segment, freed by the writer later
            ov = _Seg(f"{self.name}_ov{seq}", len(data), create=True)
            ov.buf[: len(data)] = data
            name = ov.name.encode()
            self.shm.buf[off:off + len(name)] = name
            h[1] = -len(name)
            self._overflow = getattr(self, "_overflow", [])
            self._overflow.append((seq, ov))
        h[0] = seq  # publish
        self._hdr[0] = seq
        self._seq = seq
        ovs = getattr(self, "_overflow", None)
        if ovs:
            done = int(acks.min())
            keep = []
            for s, ov in ovs:
                if s <= done:
                    ov.close()
                    ov.unlink()
                else:
                    keep.append((s, ov))
            self._overflow = keep

    # ------------------------------------------------------------------ reader
    def recv(self, timeout: Optional[float] = None) -> Any:
        assert self.reader_index >= 0
        seq = self._next
        slot = seq % self.num_slots
        h = self._slot_hdr(slot)
        self._spin(lambda: int(h[0]) == seq, timeout)
        n = int(h[1])
        off = self._slot_off(slot) + _HDR
        if n >= 0:
            obj = pickle.loads(bytes(self.shm.buf[off:off + n]))
        else:
            name = bytes(self.shm.buf[off:off - n]).decode()
            ov = _Seg(name)
            try:
                obj = pickle.loads(bytes(ov.buf))
            finally:
                ov.close()
        self._hdr[1 + self.reader_index] = seq
        self._next = seq + 1
        return obj

    def close(self):
        if self.shm is None:
            return
        self._hdr = None
        for _, ov in getattr(self, "_overflow", []):
            ov.close()
            ov.unlink()
        self._overflow = []
        self.shm.close()
        if self.owner:
            self.shm.unlink()
        self.shm = None
