"""ctypes binding to libllama3hip.so (C ABI: include/llama3hip.h).

This is the only module that touches the native library.  It has no CPU
fallback: if the shared library is missing, ``lib()`` raises, and every device
entry point raises ``RuntimeError(l3_last_error())`` on a non-zero return.
Loading the library needs no GPU (it only resolves symbols); calling a compute
entry point without a HIP device fails loudly.
"""

import ctypes
import os
import re
from typing import List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# L3_LIB_PATH: another build of the same library (kernel A/B runs in one box call, tools/ab_lib.sh);
# the product always loads the in-tree build
LIB_PATH = os.environ.get("L3_LIB_PATH") or os.path.join(HERE, "csrc", "libllama3hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "llama3hip.h")

# weight kinds / kernel ids (mirror the enums in include/llama3hip.h)
W_EMBED, W_Q, W_K, W_V, W_O, W_GATE, W_UP, W_DOWN = range(8)
W_ATTN_NORM, W_FFN_NORM, W_FINAL_NORM, W_LM_HEAD = 8, 9, 10, 11
KERNELS = ["embed", "qkv", "attn", "oproj", "gateup", "down", "lmhead", "argmax", "gather"]


class Dims(ctypes.Structure):
    _fields_ = [
        ("dim", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("n_heads", ctypes.c_int32),
        ("n_kv_heads", ctypes.c_int32),
        ("vocab_size", ctypes.c_int32),
        ("hidden_dim", ctypes.c_int32),
        ("max_seq_len", ctypes.c_int32),
        ("max_batch_size", ctypes.c_int32),
        ("norm_eps", ctypes.c_float),
    ]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_SZ = ctypes.c_size_t
_F = ctypes.c_float

_SIGNATURES = {
    "l3_last_error": (ctypes.c_char_p, []),
    "l3_device_count": (ctypes.c_int, [_P]),
    "l3_version": (ctypes.c_int, [_P, _P]),
    "l3_source_hash": (ctypes.c_char_p, []),
    "l3_host_alloc": (ctypes.c_int, [_SZ, _P]),
    "l3_host_free": (ctypes.c_int, [_P]),
    "l3_create": (ctypes.c_int, [_I32, _P, _P]),
    "l3_destroy": (ctypes.c_int, [_P]),
    "l3_upload_weight": (ctypes.c_int, [_P, _I32, _I32, _P, _I64, _I64]),
    "l3_finalize": (ctypes.c_int, [_P]),
    "l3_reset_cache": (ctypes.c_int, [_P]),
    "l3_forward_host": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P]),
    "l3_forward_dev": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P]),
    "l3_greedy_step_host": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P, _P]),
    "l3_layer_forward_host": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, _I32, _P]),
    "l3_greedy_generate_host": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P]),
    "l3_greedy_generate_values_host": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P, _P]),
    "l3_attention_forward_host": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, _I32, _P]),
    "l3_op_softmax_host": (ctypes.c_int, [_P, _P, _I64, _I64, _P]),
    "l3_op_argmax_host": (ctypes.c_int, [_P, _P, _I64, _I64, _P]),
    "l3_op_silu_host": (ctypes.c_int, [_P, _P, _I64, _P]),
    "l3_op_rmsnorm_host": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _F, _P]),
    "l3_op_rope_host": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _I32, _P, _P, _P]),
    "l3_op_ffn_host": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _P, _P, _P, _P]),
    "l3_op_linear_host": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _P, _P]),
    "l3_dev_alloc": (ctypes.c_int, [_P, _SZ, _P]),
    "l3_dev_free": (ctypes.c_int, [_P, _P]),
    "l3_h2d": (ctypes.c_int, [_P, _P, _P, _SZ]),
    "l3_d2h": (ctypes.c_int, [_P, _P, _P, _SZ]),
    "l3_synchronize": (ctypes.c_int, [_P]),
    "l3_set_batch_split": (ctypes.c_int, [_P, _I32, _I64]),
    "l3_set_gemm_x6": (ctypes.c_int, [_P, _I32]),
    "l3_set_last_layer_rows": (ctypes.c_int, [_P, _I32]),
    "l3_kernel_timing": (ctypes.c_int, [_P, _I32]),
    "l3_kernel_stats": (ctypes.c_int, [_P, _P, _P]),
    "l3_decode_stats": (ctypes.c_int, [_P, _P, _P]),
    "l3_decode_persistent": (ctypes.c_int, [_P, _P]),
    "l3_decode_recoveries": (ctypes.c_int, [_P, _P]),
    "l3_set_decode_horizon": (ctypes.c_int, [_P, _I32]),
    "l3_comm_unique_id": (ctypes.c_int, [_P]),
    "l3_comm_init": (ctypes.c_int, [_P, _I32, _I32, _P]),
    "l3_comm_gather_logits": (ctypes.c_int, [_P, _P, _P, _P, _I32]),
    "l3_comm_gather_argmax": (ctypes.c_int, [_P, _P, _P, _P, _I32]),
    "l3_comm_barrier": (ctypes.c_int, [_P]),
    "l3_comm_allreduce_max": (ctypes.c_int, [_P, _P]),
    "l3_comm_info": (ctypes.c_int, [_P, _P, _P, _P, _P, _I64]),
    "l3_comm_set_overlap": (ctypes.c_int, [_P, _I32]),
    "l3_group_create": (ctypes.c_int, [_I32, _P, _P, _P]),
    "l3_group_destroy": (ctypes.c_int, [_P]),
    "l3_group_context": (ctypes.c_int, [_P, _I32, _P]),
    "l3_group_upload_weight": (ctypes.c_int, [_P, _I32, _I32, _P, _I64, _I64]),
    "l3_group_finalize": (ctypes.c_int, [_P]),
    "l3_group_forward_host": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P]),
    "l3_group_forward_dev": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P]),
    "l3_group_greedy_step_host": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P]),
    "l3_group_synchronize": (ctypes.c_int, [_P]),
    "l3_device_check_counts": (ctypes.c_int, [_P, _P, _P]),
    "l3_device_check_selftest": (ctypes.c_int, [_P]),
}

BUSID_LEN = 16  # L3_BUSID_LEN

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load the HIP library (built by ``__graft_entry__.build()`` / ``make -C csrc``)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libllama3hip.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        so = ctypes.CDLL(LIB_PATH)
        other = bool(os.environ.get("L3_LIB_PATH"))  # an older A/B build may lack newer entry points
        for name, (res, args) in _SIGNATURES.items():
            if other and not hasattr(so, name):
                continue
            fn = getattr(so, name)
            fn.restype = res
            fn.argtypes = args
        _lib = so
    return _lib


def header_symbols() -> List[str]:
    """Every function the public header declares (used by the ABI test)."""
    with open(HEADER) as f:
        text = f.read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(l3_\w+)\s*\(", text, re.M)))


def check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError("libllama3hip: " + lib().l3_last_error().decode(errors="replace"))


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def version() -> str:
    """Library version; bumped whenever a hot kernel changes (keys profile artifacts)."""
    major, minor = ctypes.c_int32(0), ctypes.c_int32(0)
    check(lib().l3_version(ctypes.byref(major), ctypes.byref(minor)))
    return f"{major.value}.{minor.value}"


def source_hash() -> str:
    """sha256 prefix of the sources the loaded library was built from (keys profiles)."""
    return lib().l3_source_hash().decode()


class PinnedPool:
    """Page-locked host buffers handed out as NumPy arrays (``l3_host_alloc``).

    The library's host-path copies (logits D2H of ``Llama.__call__``) run as DMA at PCIe
    rate into such a buffer instead of through a pageable bounce.  The array owns its
    block through a ctypes buffer object; once the array and every view of it are gone the
    block returns to a free list and the next call of the same size reuses it (at most
    ``keep`` free blocks are kept, the rest are freed).

    Bounded: at most ``max_bytes`` are page-locked at once (blocks handed out plus cached); a
    request beyond that, or smaller than ``min_bytes`` (where pinning buys nothing), gets an
    ordinary ``np.empty`` array instead, so a caller that keeps many results never pins
    unbounded host memory."""

    def __init__(self, keep: int = 4, max_bytes: int = 1 << 30, min_bytes: int = 1 << 16):
        import threading

        self.keep = keep
        self.max_bytes = max_bytes
        self.min_bytes = min_bytes
        self._free = {}  # nbytes -> [address]
        self._pinned = 0  # bytes page-locked now: handed out + cached
        self._lock = threading.Lock()

    def empty(self, shape, dtype) -> np.ndarray:
        import weakref

        dtype = np.dtype(dtype)
        n = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
        nb = max(n, 64)
        if nb < self.min_bytes:
            return np.empty(shape, dtype)
        with self._lock:
            blocks = self._free.get(nb)
            addr = blocks.pop() if blocks else None
            if addr is None:
                if self._pinned + nb > self.max_bytes:
                    return np.empty(shape, dtype)
                self._pinned += nb  # reserved before the allocation
        if addr is None:
            p = ctypes.c_void_p()
            try:
                check(lib().l3_host_alloc(nb, ctypes.byref(p)))
            except Exception:
                with self._lock:
                    self._pinned -= nb
                raise
            addr = p.value
        holder = (ctypes.c_char * nb).from_address(addr)
        weakref.finalize(holder, self._release, addr, nb)
        return np.frombuffer(holder, dtype=dtype, count=n // dtype.itemsize).reshape(shape)

    def _release(self, addr: int, nb: int) -> None:
        with self._lock:
            blocks = self._free.setdefault(nb, [])
            if len(blocks) < self.keep:
                blocks.append(addr)
                return
            self._pinned -= nb
        lib().l3_host_free(addr)

    @property
    def pinned_bytes(self) -> int:
        return self._pinned

    def clear(self) -> None:
        """Free every cached block (arrays still alive are freed when dropped)."""
        with self._lock:
            blocks = [(a, nb) for nb, v in self._free.items() for a in v]
            self._free.clear()
            self.keep = 0
            self._pinned -= sum(nb for _, nb in blocks)
        for addr, _ in blocks:
            lib().l3_host_free(addr)


pinned = PinnedPool()


def device_count() -> int:
    n = ctypes.c_int32(0)
    check(lib().l3_device_count(ctypes.byref(n)))
    return n.value


class Context:
    """Owns one device context (weights, KV caches, workspace) on one GPU."""

    def __init__(self, dims: Dims, device: int = 0):
        self._h = ctypes.c_void_p()
        check(lib().l3_create(device, ctypes.byref(dims), ctypes.byref(self._h)))
        self.dims = dims
        self.device = device
        self._owned = True

    @classmethod
    def _member(cls, handle: ctypes.c_void_p, dims: Dims, device: int, group) -> "Context":
        """A group member's context: owned by the group (never destroyed through this object,
        which keeps the group alive)."""
        c = cls.__new__(cls)
        c._h, c.dims, c.device, c._owned, c._group = handle, dims, device, False, group
        return c

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h and getattr(self, "_owned", True):
            lib().l3_destroy(self._h)
        self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- weights ----
    def upload(self, layer: int, kind: int, w: np.ndarray) -> None:
        a = np.ascontiguousarray(w, dtype=np.float32)
        rows, cols = (1, a.shape[0]) if a.ndim == 1 else a.shape
        check(lib().l3_upload_weight(self._h, layer, kind, ptr(a), rows, cols))

    def finalize(self) -> None:
        check(lib().l3_finalize(self._h))

    def reset_cache(self) -> None:
        check(lib().l3_reset_cache(self._h))

    # ---- forward ----
    def forward(self, ids: np.ndarray, start_pos: int) -> np.ndarray:
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        B, L = ids.shape
        out = pinned.empty((B, self.dims.vocab_size), np.float32)  # DMA target of the D2H
        check(lib().l3_forward_host(self._h, ptr(ids), B, L, start_pos, ptr(out)))
        return out

    def greedy_step(self, ids: np.ndarray, start_pos: int, want_logits: bool = False):
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        B, L = ids.shape
        nxt = np.empty(B, np.int64)
        logits = pinned.empty((B, self.dims.vocab_size), np.float32) if want_logits else None
        check(lib().l3_greedy_step_host(self._h, ptr(ids), B, L, start_pos, ptr(nxt),
                                        ptr(logits) if logits is not None else None))
        return nxt, logits

    def greedy_generate(self, ids: np.ndarray, max_new_tokens: int, values: bool = False):
        """The device-side greedy loop: ids [B, max_new_tokens - L]; with ``values`` also each
        step's winning logit (fp32, same shape) — the value the step's argmax picked."""
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        B, L = ids.shape
        out = np.empty((B, max(0, max_new_tokens - L)), np.int64)
        if not values:
            check(lib().l3_greedy_generate_host(self._h, ptr(ids), B, L, max_new_tokens, ptr(out)))
            return out
        vals = np.empty(out.shape, np.float32)
        check(lib().l3_greedy_generate_values_host(self._h, ptr(ids), B, L, max_new_tokens, ptr(out), ptr(vals)))
        return out, vals

    def layer_forward(self, layer: int, x: np.ndarray, start_pos: int) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        B, L, _ = x.shape
        out = np.empty_like(x)
        check(lib().l3_layer_forward_host(self._h, layer, ptr(x), B, L, start_pos, ptr(out)))
        return out

    def attention_forward(self, layer: int, x: np.ndarray, start_pos: int) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        B, L, _ = x.shape
        out = np.empty_like(x)
        check(lib().l3_attention_forward_host(self._h, layer, ptr(x), B, L, start_pos, ptr(out)))
        return out

    # ---- device buffers (bench) ----
    def alloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        check(lib().l3_dev_alloc(self._h, nbytes, ctypes.byref(p)))
        return p.value

    def free(self, p: int) -> None:
        check(lib().l3_dev_free(self._h, p))

    def h2d(self, dst: int, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a)
        check(lib().l3_h2d(self._h, dst, ptr(a), a.nbytes))

    def d2h(self, a: np.ndarray, src: int) -> np.ndarray:
        check(lib().l3_d2h(self._h, ptr(a), src, a.nbytes))
        return a

    def forward_dev(self, ids_dev: int, B: int, L: int, start_pos: int, logits_dev: int) -> None:
        check(lib().l3_forward_dev(self._h, ids_dev, B, L, start_pos, logits_dev))

    def set_batch_split(self, parts: int, min_tokens: int = 8192) -> None:
        """Run a model forward as `parts` batch-row ranges on their own streams (extension;
        results bit-identical for any split, default 2)."""
        check(lib().l3_set_batch_split(self._h, int(parts), int(min_tokens)))

    def set_last_layer_rows(self, all_rows: bool) -> None:
        """Extension: False (default) runs the last block's attention / O-proj / FFN on each
        sequence's last position only (l3_set_last_layer_rows); True, every position."""
        check(lib().l3_set_last_layer_rows(self._h, int(bool(all_rows))))

    def set_gemm_x6(self, on: bool) -> None:
        """Extension (l3_set_gemm_x6): the prefill projections on the x6 kernel — fp32 operands
        cut exactly into three bf16 pieces, six bf16 MFMA products per fp32 product (error
        against fp64 at or below the fp32 MFMA kernel's); off (default) frees the pieces."""
        check(lib().l3_set_gemm_x6(self._h, int(bool(on))))

    def synchronize(self) -> None:
        check(lib().l3_synchronize(self._h))

    def kernel_timing(self, enable, kernels=None) -> None:
        """Record HIP events around launches (all kernels, or only the named ones)."""
        mask = 0
        if enable:
            names = KERNELS if kernels is None else kernels
            for k in names:
                mask |= 1 << KERNELS.index(k)
        check(lib().l3_kernel_timing(self._h, mask))

    def kernel_stats(self) -> dict:
        ms = np.zeros(len(KERNELS), np.float64)
        cnt = np.zeros(len(KERNELS), np.int64)
        check(lib().l3_kernel_stats(self._h, ptr(ms), ptr(cnt)))
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(KERNELS)}

    def set_decode_horizon(self, end_pos: int) -> None:
        """Lazy decode runs ahead of the caller on the device; never at positions >= end_pos."""
        check(lib().l3_set_decode_horizon(self._h, int(end_pos)))

    def decode_persistent(self) -> bool:
        """True when the captured batch-1 decode step is the persistent one-launch kernel."""
        v = ctypes.c_int32(0)
        check(lib().l3_decode_persistent(self._h, ctypes.byref(v)))
        return bool(v.value)

    def decode_recoveries(self) -> int:
        """Persistent decode steps that gave up on a hand-off and were re-run on the graph path."""
        v = ctypes.c_int64(0)
        check(lib().l3_decode_recoveries(self._h, ctypes.byref(v)))
        return int(v.value)

    def device_check_counts(self):
        """(enabled, counts): the device bounds-check counters (check build, L3_LIB_PATH =
        libllama3hip_check.so) since the last call — K / V slot, attention keys, token id."""
        n = np.zeros(4, np.uint32)
        en = ctypes.c_int32(0)
        check(lib().l3_device_check_counts(self._h, n.ctypes.data_as(ctypes.c_void_p), ctypes.byref(en)))
        return bool(en.value), {"kv_slot": int(n[0]), "attn_keys": int(n[1]), "token_id": int(n[2])}

    def device_check_selftest(self) -> None:
        """One recorded violation of each check class (check build; a no-op in the release one)."""
        check(lib().l3_device_check_selftest(self._h))

    def decode_stats(self) -> dict:
        """Decode steps served by graph replay, and of those by a speculative step."""
        v = np.zeros(2, np.int64)
        check(lib().l3_decode_stats(self._h, ptr(v[0:1]), ptr(v[1:2])))
        return {"graph_steps": int(v[0]), "speculative_hits": int(v[1])}

    # ---- RCCL ----
    def comm_init(self, nranks: int, rank: int, uid: bytes) -> None:
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(lib().l3_comm_init(self._h, nranks, rank, buf))
        self.nranks, self.rank = nranks, rank

    def _rows(self, rows_per_rank) -> np.ndarray:
        rows = np.ascontiguousarray(rows_per_rank, dtype=np.int64)
        n = getattr(self, "nranks", None)
        if n is None:
            raise RuntimeError("communicator not initialised (comm_init)")
        if rows.shape != (n,):
            raise ValueError(f"rows_per_rank has {rows.size} entries, the communicator {n} ranks")
        return rows

    def gather_logits(self, src_dev: int, dst_dev: Optional[int], rows_per_rank, root: int = 0):
        rows = self._rows(rows_per_rank)
        check(lib().l3_comm_gather_logits(self._h, src_dev, dst_dev or 0, ptr(rows), root))

    def gather_argmax(self, src_dev: int, dst_dev: Optional[int], rows_per_rank, root: int = 0):
        """Greedy ids only: each rank's argmax over its logits rows, int32 ids gathered to
        ``dst_dev`` [sum rows] on the root (SURVEY 8(e) option)."""
        rows = self._rows(rows_per_rank)
        check(lib().l3_comm_gather_argmax(self._h, src_dev, dst_dev or 0, ptr(rows), root))

    def comm_info(self, gather_busids: bool = True) -> dict:
        """What RCCL reports for this rank (ncclCommCount / ncclCommUserRank /
        ncclCommCuDevice) and, with ``gather_busids`` (collective: every rank calls it), every
        rank's PCI bus id in rank order."""
        n, r, d = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
        cap = getattr(self, "nranks", 1) if gather_busids else 0
        buf = ctypes.create_string_buffer(BUSID_LEN * max(cap, 1))
        check(lib().l3_comm_info(self._h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d),
                                 buf if gather_busids else None, cap))
        out = {"nranks": n.value, "rank": r.value, "device": d.value}
        if gather_busids:
            raw = buf.raw
            out["busids"] = [raw[i * BUSID_LEN:(i + 1) * BUSID_LEN].split(b"\0")[0].decode()
                             for i in range(n.value)]
        return out

    def set_comm_overlap(self, on: bool) -> None:
        """The overlapped logits gather (next forward's second batch part runs during it)."""
        check(lib().l3_comm_set_overlap(self._h, int(bool(on))))

    def comm_barrier(self) -> None:
        check(lib().l3_comm_barrier(self._h))

    def comm_max(self, x: float) -> float:
        v = ctypes.c_double(x)
        check(lib().l3_comm_allreduce_max(self._h, ctypes.byref(v)))
        return v.value

    # ---- ops ----
    def op_softmax(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        y = np.empty_like(x)
        n = x.shape[-1]
        check(lib().l3_op_softmax_host(self._h, ptr(x), x.size // n, n, ptr(y)))
        return y

    def op_argmax(self, x: np.ndarray) -> np.ndarray:
        """argmax over the last axis (np.argmax tie-break, NaN first); int32 of x.shape[:-1]."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        n = x.shape[-1]
        out = np.empty(x.shape[:-1], np.int32)
        check(lib().l3_op_argmax_host(self._h, ptr(x), x.size // n, n, ptr(out)))
        return out

    def op_silu(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        y = np.empty_like(x)
        check(lib().l3_op_silu_host(self._h, ptr(x), x.size, ptr(y)))
        return y

    def op_rmsnorm(self, x: np.ndarray, w: np.ndarray, eps: float) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        w = np.ascontiguousarray(w, dtype=np.float32)
        y = np.empty_like(x)
        n = x.shape[-1]
        check(lib().l3_op_rmsnorm_host(self._h, ptr(x), ptr(w), x.size // n, n, eps, ptr(y)))
        return y

    def op_rope(self, x: np.ndarray, cos_t: np.ndarray, sin_t: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        c = np.ascontiguousarray(cos_t, dtype=np.float32)
        s = np.ascontiguousarray(sin_t, dtype=np.float32)
        B, L, nh, hd = x.shape
        y = np.empty_like(x)
        check(lib().l3_op_rope_host(self._h, ptr(x), B, L, nh, hd, ptr(c), ptr(s), ptr(y)))
        return y

    def op_linear(self, x: np.ndarray, w: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        w = np.ascontiguousarray(w, dtype=np.float32)
        K = x.shape[-1]
        N = w.shape[0]
        y = np.empty(x.shape[:-1] + (N,), np.float32)
        check(lib().l3_op_linear_host(self._h, ptr(x), x.size // K, K, N, ptr(w), ptr(y)))
        return y

    def op_ffn(self, x: np.ndarray, wg: np.ndarray, wu: np.ndarray, wd: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        D = x.shape[-1]
        FD = wg.shape[0]
        y = np.empty_like(x)
        wg, wu, wd = (np.ascontiguousarray(a, dtype=np.float32) for a in (wg, wu, wd))
        check(lib().l3_op_ffn_host(self._h, ptr(x), x.size // D, D, FD, ptr(wg), ptr(wu), ptr(wd),
                                   ptr(y)))
        return y


def member_rows(B: int, n: int, i: int) -> int:
    """Rows of group member i (of n) in a batch of B: global rows i, i + n, i + 2n, ... — the
    l3_group row mapping (row r on member r % n as its local row r // n), which does not depend
    on B, so a row's KV cache stays on one device across calls of any batch size."""
    if n <= 0 or not 0 <= i < n:
        raise ValueError(f"bad member {i} of {n}")
    return (B - i + n - 1) // n if B > i else 0


class Group:
    """One process driving ``devices`` (l3_group_*, include/llama3hip.h): one context per
    device, RCCL communicators from ncclCommInitAll, batch row r on member r % n (its local
    row r // n).  Same upload / finalize / forward / greedy_step surface as ``Context``."""

    def __init__(self, dims: Dims, devices):
        devs = np.ascontiguousarray(list(devices), dtype=np.int32)
        if devs.ndim != 1 or devs.size == 0:
            raise ValueError("devices must be a non-empty list of device ordinals")
        self._h = ctypes.c_void_p()
        check(lib().l3_group_create(int(devs.size), ptr(devs), ctypes.byref(dims), ctypes.byref(self._h)))
        self.dims = dims
        self.devices = [int(x) for x in devs]
        self.n = len(self.devices)
        local = Dims.from_buffer_copy(dims)
        local.max_batch_size = -(-dims.max_batch_size // self.n)
        self.members = []
        for i, dv in enumerate(self.devices):
            h = ctypes.c_void_p()
            check(lib().l3_group_context(self._h, i, ctypes.byref(h)))
            m = Context._member(h, local, dv, self)
            m.nranks, m.rank = self.n, i  # its communicator (ncclCommInitAll), used via the group
            self.members.append(m)

    def close(self):
        if self._h:
            for m in self.members:
                m._h = ctypes.c_void_p()
            lib().l3_group_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def rows(self, B: int, i: int) -> int:
        """Rows of member i in a batch of B (rows i, i + n, ...)."""
        return member_rows(B, self.n, i)

    def upload(self, layer: int, kind: int, w: np.ndarray) -> None:
        a = np.ascontiguousarray(w, dtype=np.float32)
        rows, cols = (1, a.shape[0]) if a.ndim == 1 else a.shape
        check(lib().l3_group_upload_weight(self._h, layer, kind, ptr(a), rows, cols))

    def finalize(self) -> None:
        check(lib().l3_group_finalize(self._h))

    def forward(self, ids: np.ndarray, start_pos: int) -> np.ndarray:
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        B, L = ids.shape
        out = pinned.empty((B, self.dims.vocab_size), np.float32)
        check(lib().l3_group_forward_host(self._h, ptr(ids), B, L, start_pos, ptr(out)))
        return out

    def forward_dev(self, ids_dev, B: int, L: int, start_pos: int, logits_dev: int) -> None:
        """ids_dev: one device pointer per member (its rows, int32); logits_dev on member 0."""
        arr = (ctypes.c_void_p * self.n)(*[ctypes.c_void_p(p or 0) for p in ids_dev])
        check(lib().l3_group_forward_dev(self._h, arr, B, L, start_pos, logits_dev))

    def greedy_step(self, ids: np.ndarray, start_pos: int, want_logits: bool = False):
        if want_logits:
            raise NotImplementedError("Group.greedy_step returns ids only")
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        B, L = ids.shape
        nxt = np.empty(B, np.int64)
        check(lib().l3_group_greedy_step_host(self._h, ptr(ids), B, L, start_pos, ptr(nxt)))
        return nxt, None

    def set_decode_horizon(self, end_pos: int) -> None:
        self.members[0].set_decode_horizon(end_pos)

    def synchronize(self) -> None:
        check(lib().l3_group_synchronize(self._h))

    def _single(self) -> Context:
        if self.n != 1:
            raise RuntimeError("a per-block call on a multi-device Llama: its KV cache rows are spread "
                               "over the devices; build a TransformerBlock from the weights instead")
        return self.members[0]

    def layer_forward(self, layer: int, x: np.ndarray, start_pos: int) -> np.ndarray:
        return self._single().layer_forward(layer, x, start_pos)

    def attention_forward(self, layer: int, x: np.ndarray, start_pos: int) -> np.ndarray:
        return self._single().attention_forward(layer, x, start_pos)


def launch_key() -> str:
    """Key of the RCCL-id hand-off file: equal on every rank of one launch, different for every
    launch — torchrun's run id (TORCHELASTIC_RUN_ID; "none" under the default static rendezvous,
    so not unique alone), the launcher's pid (torchrun's agent is the parent of every rank it
    starts) and MASTER_PORT.  A launcher that sets L3_LAUNCH_KEY (bench.py's spawn_ranks) names
    the launch itself."""
    own = os.environ.get("L3_LAUNCH_KEY")
    if own:
        return own
    run = os.environ.get("TORCHELASTIC_RUN_ID") or "local"
    return f"{run}_{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}"


def remove_unique_id(key: str) -> None:
    """Rank 0, once every rank has joined the communicator (ncclCommInitRank is collective, so
    every rank has read the id by then): drop the hand-off file."""
    try:
        os.remove(os.path.join("/tmp", f"l3_rccl_uid_{key}"))
    except OSError:
        pass


def exchange_unique_id(rank: int, world: int, key: str, timeout_s: float = 120.0) -> bytes:
    """Ship the 128-byte RCCL id from rank 0 to the other ranks of ONE node through an
    atomically renamed file in /tmp (no PyTorch / gloo needed).  ``key`` must be unique per
    launch and equal on all ranks (e.g. launcher pid + MASTER_PORT)."""
    import time

    path = os.path.join("/tmp", f"l3_rccl_uid_{key}")
    if rank == 0:
        uid = comm_unique_id()
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.time()
    while True:
        try:
            with open(path, "rb") as f:
                uid = f.read()
            if len(uid) == 128:
                return uid
        except FileNotFoundError:
            pass
        if time.time() - t0 > timeout_s:
            raise RuntimeError(f"timed out waiting for the RCCL id at {path}")
        time.sleep(0.01)


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * 128)()
    check(lib().l3_comm_unique_id(buf))
    return bytes(buf)


_op_ctx = {}


def op_context(device: int = 0) -> Context:
    """Shared op-only context (n_layers = 0) used by the module-level ops."""
    if device not in _op_ctx:
        d = Dims(dim=64, n_layers=0, n_heads=1, n_kv_heads=1, vocab_size=1, hidden_dim=32,
                 max_seq_len=1, max_batch_size=1, norm_eps=1e-6)
        _op_ctx[device] = Context(d, device)
    return _op_ctx[device]
