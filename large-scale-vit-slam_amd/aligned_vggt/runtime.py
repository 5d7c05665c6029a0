"""Host-side runtime for the HIP hot path: packed-weight cache and device
workspaces.

* Weights stay fp32 ``nn.Parameter``s with the reference module-tree names
  (state-dict compatible, featureAligned_vggt.py:16-32); the bf16 operand
  copies the MFMA kernels read are derived lazily and re-derived whenever the
  parameter changes (tracked by ``_version`` / data pointer).
* Activations live in per-device workspaces sized for the largest chunk seen
  (288 GB of HBM per MI355X: buffers are kept, never freed per chunk -- the
  reference instead calls ``torch.cuda.empty_cache()`` every chunk,
  featureAligned_vggt.py:82).
"""
from __future__ import annotations

import contextlib
import os
import threading
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn


def _pkey(*ts):
    return tuple((t.data_ptr(), t._version, t.device) if t is not None else None for t in ts)


def pack_linear(lin: nn.Linear, k_pad: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """(W bf16 [N, K(+pad)], bias rounded through bf16 as fp32 [N]).

    Under the reference's bf16-mixed autocast nn.Linear casts weight AND bias
    to bf16; the rounded bias is kept in fp32 for the epilogue add."""
    w, b = lin.weight, lin.bias
    key = _pkey(w, b) + (k_pad,)
    c = lin.__dict__.get("_mi355x_pack")
    if c is None or c[0] != key:
        wq = w.detach().reshape(w.shape[0], -1).to(torch.bfloat16)
        if k_pad:
            wq = torch.nn.functional.pad(wq, (0, k_pad))
        bq = (b.detach().to(torch.bfloat16).float() if b is not None
              else torch.zeros(w.shape[0], device=w.device, dtype=torch.float32))
        c = (key, wq.contiguous(), bq.contiguous())
        lin.__dict__["_mi355x_pack"] = c
    return c[1], c[2]


def f32_param(mod: nn.Module, name: str, fill: Optional[float] = None, n: int = 0) -> torch.Tensor:
    """fp32 contiguous view of a parameter (or a cached constant vector)."""
    p = getattr(mod, name, None)
    if p is None:
        key = ("_mi355x_const", name, fill, n)
        c = mod.__dict__.get(key[0] + name)
        dev = next(mod.parameters()).device
        if c is None or c.device != dev or c.numel() != n:
            c = torch.full((n,), fill, device=dev, dtype=torch.float32)
            mod.__dict__[key[0] + name] = c
        return c
    return p.detach().float().contiguous() if p.dtype != torch.float32 or not p.is_contiguous() else p.detach()


_SCOPE = threading.local()


@contextlib.contextmanager
def private_scratch(store: dict):
    """Route every grow-only scratch lookup (Workspace, the split-K and
    training-reduction slabs of _native) made inside the block to ``store``
    instead of the shared per-(device, stream) tables.  A HIP graph's capture
    and its warm-ups run inside one, with a store the graph object owns: the
    pointers the graph bakes in then belong to it alone.  Shared tables are
    keyed by stream, and torch hands capture streams out of a small pool, so a
    later graph -- or eager work -- on the same pool stream could otherwise
    grow (re-allocate) a buffer an earlier graph still replays into."""
    prev = getattr(_SCOPE, "store", None)
    _SCOPE.store = store
    try:
        yield store
    finally:
        _SCOPE.store = prev


def scratch_table(shared: dict, kind: str) -> dict:
    """The table scratch of ``kind`` lives in: the active private store's, else ``shared``."""
    st = getattr(_SCOPE, "store", None)
    return shared if st is None else st.setdefault(kind, {})


class Workspace:
    """Named, grow-only device buffers: one set per (device, stream), so work
    queued on two streams at once (the multi-GPU pipeline aligns chunk i on a
    side stream while the compute stream encodes chunk i + W) never shares a
    scratch buffer; a captured graph's own set inside ``private_scratch``."""

    _per_device: Dict[tuple, "Workspace"] = {}

    def __init__(self, device):
        self.device = device
        self.bufs: Dict[str, torch.Tensor] = {}

    @classmethod
    def get(cls, device) -> "Workspace":
        device = torch.device(device)
        if device.type == "cuda":
            if device.index is None:
                device = torch.device("cuda", torch.cuda.current_device())
            key = (device, torch.cuda.current_stream(device).stream_id)
        else:
            key = (device, 0)
        table = scratch_table(cls._per_device, "workspace")
        ws = table.get(key)
        if ws is None:
            ws = table[key] = Workspace(device)
        return ws

    def buf(self, name: str, rows: int, cols: int, dtype=torch.float32) -> torch.Tensor:
        t = self.bufs.get(name)
        need = rows * cols
        if t is None or t.dtype != dtype or t.numel() < need:
            t = torch.zeros(need, device=self.device, dtype=dtype)
            self.bufs[name] = t
        return t[:need].view(rows, cols)


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# module-dict caches derived from parameter VALUES (bf16 packs, transposes,
# concatenations); everything else cached on modules (RoPE tables, positions,
# constant vectors) depends on shapes only
WEIGHT_CACHES = ("_mi355x_pack", "_mi355x_wt", "_mi355x_kv")


def drop_weight_caches(module: nn.Module) -> None:
    """Forget every operand derived from a parameter's values, so the next
    forward re-derives it (a HIP graph captured after this records the
    re-derivation and repeats it on every replay, after each optimizer step)."""
    for m in module.modules():
        for k in [k for k in m.__dict__ if k.startswith(WEIGHT_CACHES)]:
            del m.__dict__[k]


class GraphedStep:
    """One HIP graph for a launch-bound step.

    The alignment-head training forward + backward is ~2,000 small kernels
    per step (two chunks, 48 checkpoint-style block Functions, their HIP
    backward kernels, the fused AdamW aside); issued eagerly through Python
    and ctypes the device idles between many of them.  Captured once, the
    whole sequence is replayed by one hipGraphLaunch.

    ``fn`` must read only tensors whose storage stays put between calls
    (parameters, resident inputs updated in place) and must not synchronise
    with the host.  It runs ``warmup`` times eagerly on the capture stream
    (settles workspace sizes and shape-keyed caches: RoPE tables, device
    position vectors), then once under capture; the weight-derived caches of
    ``modules`` are dropped first so the capture records their re-derivation
    (parameters change in place between replays).  ``__call__`` replays and
    returns the captured call's outputs (static tensors, overwritten by each
    replay).  Gradients written by a captured backward are the static buffers
    the capture allocated: do not ``zero_grad(set_to_none=True)`` between
    replays (the captured step re-zeroes them itself)."""

    def __init__(self, fn, modules=(), warmup: int = 2, device=None):
        self.fn = fn
        self.modules = list(modules)
        self.warmup = warmup
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.graph = None
        self.out = None
        self.scratch = {}  # this graph's own workspaces (private_scratch)

    def capture(self) -> None:
        if self.device.type != "cuda":
            raise RuntimeError("GraphedStep: HIP graphs need a HIP device")
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with private_scratch(self.scratch):
            with torch.cuda.stream(s):
                for _ in range(self.warmup):
                    self.fn()
            s.synchronize()
            for m in self.modules:
                drop_weight_caches(m)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self.out = self.fn()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graph = g

    def __call__(self):
        if self.graph is None:
            self.capture()
        self.graph.replay()
        return self.out


def spread_cus(ncu: int, n: int) -> list:
    """n CU indices spread over the chip so that each of the 8 XCDs gets the
    same share whether the CU-mask bits enumerate CUs XCD by XCD or
    round-robin over the XCDs: index k*(ncu/n) + (k mod 8)."""
    step = max(1, ncu // max(1, n))
    return sorted({(k * step + (k % 8)) % ncu for k in range(n)})


_HIP = None


def _hip():
    import ctypes
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
        _HIP.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
        _HIP.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
        _HIP.hipStreamCreateWithPriority.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint, ctypes.c_int]
        _HIP.hipStreamCreateWithPriority.restype = ctypes.c_int
        _HIP.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        _HIP.hipExtMallocWithFlags.restype = ctypes.c_int
        _HIP.hipFree.argtypes = [ctypes.c_void_p]
        _HIP.hipFree.restype = ctypes.c_int
        _HIP.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint,
                                              ctypes.c_uint32]
        _HIP.hipStreamWaitValue32.restype = ctypes.c_int
        _HIP.hipStreamWriteValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint]
        _HIP.hipStreamWriteValue32.restype = ctypes.c_int
        _HIP.hipStreamGetPriority.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        _HIP.hipStreamGetPriority.restype = ctypes.c_int
    return _HIP


def stream_priority(stream) -> int:
    """The HIP priority of a torch stream (lower = higher priority; the null stream's is 0)."""
    import ctypes
    p = ctypes.c_int(0)
    rc = _hip().hipStreamGetPriority(ctypes.c_void_p(stream.cuda_stream), ctypes.byref(p))
    if rc != 0:
        raise RuntimeError(f"hipStreamGetPriority failed ({rc})")
    return p.value


class EncodeGate:
    """A device-side pause for the multi-GPU pipeline's encode stream while an
    alignment runs: one 32-bit signal word (hipExtMallocWithFlags,
    hipMallocSignalMemory).  The alignment stream writes 1 when it starts a
    chunk (after its device-side waits for the baton and the chunk's encode)
    and 0 when it is done (hipStreamWriteValue32); the encode stream, at its
    yield points (`yield_point`, between transformer blocks and heads), waits
    for 0 (hipStreamWaitValue32).  An alignment therefore shares the GPU with
    at most one yield interval of encode work and then runs alone.

    Why it cannot deadlock (the rules the pipeline keeps):
      * the word goes to 1 only after the chunk's own encode has finished, and
        the alignment stream never waits on the encode stream after that;
      * no device-wide wait between begin and end: a hipDeviceSynchronize (a
        HIP graph capture's, an allocator's hipFree on an out-of-memory retry)
        issued by the host while the gate is held would wait for the paused
        encode, which waits for the end() the host has not enqueued yet.  The
        ring therefore runs ``prepare_align`` (graph capture) before begin();
      * the alignment stream has a strictly higher priority than the encode
        stream (checked before the gate is used, else the ring runs ungated):
        HIP maps priorities to separate hardware-queue pools, so with
        GPU_MAX_HW_QUEUES = 4 and more normal-priority streams than queues the
        encode's spinning wait can share a queue with other normal streams but
        never sits ahead of the alignment's begin/end writes in one queue."""

    def __init__(self, device):
        import ctypes
        self.device = torch.device(device)
        p = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            rc = _hip().hipExtMallocWithFlags(ctypes.byref(p), 8, 0x2)  # hipMallocSignalMemory: one 8-byte signal
            if rc != 0:
                raise RuntimeError(f"hipExtMallocWithFlags(hipMallocSignalMemory) failed ({rc})")
            self.ptr = p.value
            s = torch.cuda.current_stream(self.device)
            self._write(s.cuda_stream, 0)
            s.synchronize()

    def _write(self, stream: int, v: int) -> None:
        import ctypes
        rc = _hip().hipStreamWriteValue32(ctypes.c_void_p(stream), ctypes.c_void_p(self.ptr), v, 0)
        if rc != 0:
            raise RuntimeError(f"hipStreamWriteValue32 failed ({rc})")

    def begin(self, stream) -> None:
        """On the alignment stream, after its waits: the encode pauses at its next yield point."""
        self._write(stream.cuda_stream, 1)

    def end(self, stream) -> None:
        self._write(stream.cuda_stream, 0)

    def wait(self, stream: int) -> None:
        import ctypes
        rc = _hip().hipStreamWaitValue32(ctypes.c_void_p(stream), ctypes.c_void_p(self.ptr), 0, 0x1,
                                         0xFFFFFFFF)  # hipStreamWaitValueEq
        if rc != 0:
            raise RuntimeError(f"hipStreamWaitValue32 failed ({rc})")

    def close(self) -> None:
        if getattr(self, "ptr", None):
            import ctypes
            torch.cuda.synchronize(self.device)
            _hip().hipFree(ctypes.c_void_p(self.ptr))
            self.ptr = None


_GATE = threading.local()


@contextlib.contextmanager
def gated(stream, gate: "EncodeGate"):
    """Within the block, `yield_point()` calls made while `stream` is current
    enqueue a wait on `gate` (the encode stream of the pipeline's ring)."""
    prev = getattr(_GATE, "cur", None)
    _GATE.cur = (stream.cuda_stream, gate)
    try:
        yield
    finally:
        _GATE.cur = prev


# VGGT_GATE_FINE=1: also yield before the large GEMMs inside each block and before
# every DPT convolution (shorter intervals of encode work still in flight when an
# alignment starts)
_GATE_FINE = os.environ.get("VGGT_GATE_FINE", "0") == "1"


def yield_point(fine: bool = False) -> None:
    """A place in the encode (between transformer blocks, before each head)
    where a gated encode stream pauses while an alignment runs; a no-op
    otherwise.  ``fine`` points count only with VGGT_GATE_FINE=1."""
    cur = getattr(_GATE, "cur", None)
    if cur is None or (fine and not _GATE_FINE):
        return
    handle, gate = cur
    if torch.cuda.current_stream(gate.device).cuda_stream == handle:
        gate.wait(handle)


def dedicated_stream(device, priority: int = 0) -> "torch.cuda.ExternalStream":
    """A HIP stream of its own (non-blocking; not one of torch's pooled streams,
    which other users are handed too), as a torch ExternalStream -- for a
    per-stream library configuration (vggt_set_stream_config) that must apply to
    this stream's work only.  `priority` as torch.cuda.Stream's (lower = higher)."""
    import ctypes
    device = torch.device(device)
    s = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = _hip().hipStreamCreateWithPriority(ctypes.byref(s), 1, int(priority))  # hipStreamNonBlocking
    if rc != 0:
        raise RuntimeError(f"hipStreamCreateWithPriority failed ({rc})")
    return torch.cuda.ExternalStream(s.value, device=device)


def cu_masked_stream(device, exclude) -> "torch.cuda.ExternalStream":
    """A HIP stream whose kernels never run on the CUs in ``exclude``
    (hipExtStreamCreateWithCUMask), as a torch ExternalStream.  The multi-GPU
    pipeline encodes on such a stream so that the alignment recurrence's
    kernels, on their own high-priority stream, always find those CUs free
    instead of waiting behind a persistent GEMM or attention launch."""
    import ctypes
    device = torch.device(device)
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    words = [0xFFFFFFFF] * ((ncu + 31) // 32)
    if ncu % 32:
        words[-1] = (1 << (ncu % 32)) - 1
    for i in exclude:
        words[i // 32] &= ~(1 << (i % 32)) & 0xFFFFFFFF
    arr = (ctypes.c_uint32 * len(words))(*words)
    s = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = _hip().hipExtStreamCreateWithCUMask(ctypes.byref(s), len(words), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    return torch.cuda.ExternalStream(s.value, device=device)


_SHARED_STREAMS: Dict[tuple, "torch.cuda.ExternalStream"] = {}


def shared_stream(device, exclude_cus: int = 0, priority: int = 0, short_workgroups: bool = False):
    """The pipeline's dedicated streams, one per (device, configuration) for the
    life of the process: a non-blocking stream (dedicated_stream) or one masked
    off ``exclude_cus`` CUs spread over the XCDs (cu_masked_stream), registered
    once with the library (vggt_set_stream_config: the CUs its persistent grids
    may size to, short workgroups).  Shared rather than created per pipeline:
    the library has 16 configuration slots, and a stream cannot be destroyed
    while the caching allocator may still record events on it for blocks it
    handed out there (torch keeps no count of them)."""
    device = torch.device(device)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = (device, exclude_cus, priority, short_workgroups)
    s = _SHARED_STREAMS.get(key)
    if s is None:
        from . import _native as N
        cus = 0
        if exclude_cus > 0:
            ncu = torch.cuda.get_device_properties(device).multi_processor_count
            excl = spread_cus(ncu, exclude_cus)
            s = cu_masked_stream(device, excl)
            cus = ncu - len(excl)
        else:
            s = dedicated_stream(device, priority=priority)
        if cus or short_workgroups:
            N.set_stream_config(s.cuda_stream, cus, N.STREAM_SHORT_WORKGROUPS if short_workgroups else 0)
        _SHARED_STREAMS[key] = s
    return s
