"""Weight loading — drop-in for the reference's ``utils.load_parameters``.

Reference: ``utils.py:4-5`` returns ``np.load(model_path)``: a lazy ``NpzFile``
mapping from HF-style tensor names to fp32 arrays stored ``[out, in]``
row-major.  We return the same object (pickle stays disabled, NumPy's
default), so ``weight.get(name)`` and ``weight[name]`` behave identically.

``StreamingNpz`` (extension) is the ``.npz`` reader of ``Llama.__init__``: each member is
read from the file by several ``preadv`` threads into a buffer from an allocator the caller
passes — ordinary memory recycled per size (``RecyclingAlloc``) by default, page-locked
buffers from ``l3hip.PinnedPool`` with ``L3_NPZ_READER=pinned``.

``weight_names`` lists every key the forward pass reads; ``Llama.__init__`` checks them all
before it allocates anything, to fail early on a missing tensor instead of the reference's
late ``AttributeError`` on ``None.T`` (``llama3.py:133-136``).
"""

import ctypes
import os
import struct
import zipfile
from typing import Callable, List, Optional

import numpy as np


def load_parameters(model_path):
    return np.load(model_path, allow_pickle=False)


class StreamingNpz:
    """Extension: the streaming loader's view of an ``.npz``.

    ``get(name)`` reads one member straight from the file into a buffer made by
    ``alloc(shape, dtype)`` — ``np.empty`` when host copies are kept, a ``RecyclingAlloc``
    (ordinary memory, reused per size once uploaded) in ``Llama(..., keep_host_weights=False)``,
    or page-locked ``l3hip.PinnedPool`` buffers with ``L3_NPZ_READER=pinned`` (a DMA upload;
    measured slower overall) — and the bytes are copied once (page cache -> buffer,
    32 MB ``preadv`` pieces on ``threads`` threads at once) instead of three times
    (``NpzFile``: zip stream -> 256 KB chunks -> array, with a CRC-32 pass, then the runtime's
    bounce).  Stored
    (uncompressed, as ``np.savez`` writes them) little-endian fp32 C-order members take this path; any other member (compressed,
    Fortran order, another dtype, a newer ``.npy`` header) is read by ``NpzFile`` as the
    reference's ``load_parameters`` would (same values either way; the fast path skips the
    zip CRC check, the ``.npy`` header is still parsed and checked against the member size).
    Same lookup contract as the reference's mapping: ``get`` returns ``default`` for a
    missing key."""

    CHUNK = 32 << 20  # bytes per read request

    def __init__(self, model_path, alloc: Callable[[tuple, np.dtype], np.ndarray],
                 threads: int = 8):
        self.threads = max(1, min(threads, os.cpu_count() or 1))
        self._alloc = alloc
        self._zip = zipfile.ZipFile(model_path)
        self._raw = open(model_path, "rb", buffering=0)
        self._members = {zi.filename[:-4]: zi for zi in self._zip.infolist()
                         if zi.filename.endswith(".npy")}
        self._npz: Optional[np.lib.npyio.NpzFile] = None
        self._path = model_path
        self._pool = None

    def keys(self):
        return self._members.keys()

    def __contains__(self, name) -> bool:
        return name in self._members

    def __getitem__(self, name):
        out = self.get(name)
        if out is None:
            raise KeyError(name)
        return out

    def _fallback(self, name):
        if self._npz is None:
            self._npz = np.load(self._path, allow_pickle=False)
        return self._npz[name]

    def get(self, name, default=None):
        zi = self._members.get(name)
        if zi is None:
            return default
        if zi.compress_type != zipfile.ZIP_STORED:
            return self._fallback(name)
        f = self._raw
        f.seek(zi.header_offset)
        local = f.read(30)
        sig, *_, name_len, extra_len = struct.unpack("<IHHHHHIIIHH", local)
        if sig != 0x04034B50:
            raise ValueError(f"{self._path}: bad zip local header for member {zi.filename!r}")
        start = zi.header_offset + 30 + name_len + extra_len
        f.seek(start)
        version = np.lib.format.read_magic(f)
        if version == (1, 0):
            shape, fortran, dtype = np.lib.format.read_array_header_1_0(f)
        elif version == (2, 0):
            shape, fortran, dtype = np.lib.format.read_array_header_2_0(f)
        else:
            return self._fallback(name)
        if fortran or dtype != np.dtype("<f4"):
            return self._fallback(name)
        nbytes = int(np.prod(shape, dtype=np.int64)) * 4
        if f.tell() - start + nbytes != zi.file_size:
            raise ValueError(f"{self._path}: member {zi.filename!r} size does not match its header")
        out = self._alloc(tuple(shape), np.float32)
        view = memoryview(out.reshape(-1)).cast("B")
        data = f.tell()
        chunks = [(o, min(nbytes, o + self.CHUNK)) for o in range(0, nbytes, self.CHUNK)]
        if len(chunks) > 1 and self.threads > 1:
            if self._pool is None:
                from concurrent.futures import ThreadPoolExecutor

                self._pool = ThreadPoolExecutor(self.threads)
            list(self._pool.map(lambda c: self._pread(view, data, *c, zi), chunks))
        else:
            for c in chunks:
                self._pread(view, data, *c, zi)
        return out

    def _pread(self, view, data, lo, hi, zi):
        # os.preadv releases the GIL: chunks of one member are copied out of the page cache by
        # several threads at once (one thread tops out near 4.4 GB/s on the box)
        fd = self._raw.fileno()
        while lo < hi:
            n = os.preadv(fd, [view[lo:hi]], data + lo)
            if not n:
                raise ValueError(f"{self._path}: member {zi.filename!r} truncated")
            lo += n

    def close(self) -> None:
        if self._pool is not None:
            self._pool.shutdown()
            self._pool = None
        self._raw.close()
        self._zip.close()
        if self._npz is not None:
            self._npz.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RecyclingAlloc:
    """``alloc(shape, dtype)`` for ``StreamingNpz`` when the arrays are dropped after upload
    (``keep_host_weights=False``): an array's memory goes back to a per-size free list once the
    array and every view of it are gone, and the next member of that size reuses it — no fresh
    pages to fault in and no unmap per member (at most ``keep`` blocks per size are kept)."""

    def __init__(self, keep: int = 3):
        import threading

        self.keep = keep
        self._free = {}
        self._lock = threading.Lock()

    def __call__(self, shape, dtype) -> np.ndarray:
        import weakref

        dtype = np.dtype(dtype)
        n = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
        with self._lock:
            blocks = self._free.get(n)
            buf = blocks.pop() if blocks else None
        if buf is None:
            buf = np.empty(max(n, 1), np.uint8)
        # every view NumPy derives from the result points at this holder (the buffer's exporter),
        # so it outlives all of them and its finaliser is the release point
        holder = (ctypes.c_char * max(n, 1)).from_buffer(buf)
        weakref.finalize(holder, self._release, buf, n)
        return np.frombuffer(holder, dtype=dtype, count=n // dtype.itemsize).reshape(shape)

    def _release(self, buf, n) -> None:
        with self._lock:
            if len(self._free.get(n, ())) < self.keep:
                self._free.setdefault(n, []).append(buf)

    def clear(self) -> None:
        with self._lock:
            self._free.clear()
            self.keep = 0


def weight_names(n_layers: int) -> List[str]:
    names = ["model.embed_tokens.weight", "model.norm.weight", "lm_head.weight"]
    for i in range(n_layers):
        p = f"model.layers.{i}."
        names += [
            p + "self_attn.q_proj.weight",
            p + "self_attn.k_proj.weight",
            p + "self_attn.v_proj.weight",
            p + "self_attn.o_proj.weight",
            p + "mlp.gate_proj.weight",
            p + "mlp.up_proj.weight",
            p + "mlp.down_proj.weight",
            p + "input_layernorm.weight",
            p + "post_attention_layernorm.weight",
        ]
    return names
