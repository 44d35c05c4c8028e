"""Small helpers shared by the op wrappers."""
from __future__ import annotations

import contextlib

import torch

from .. import _native

BF16 = torch.bfloat16
F32 = torch.float32


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


class IntOut:
    """A C int the native side can write (passed as its address)."""

    def __init__(self):
        import ctypes
        self._v = ctypes.c_int(0)
        self.addr = ctypes.addressof(self._v)

    @property
    def value(self):
        return self._v.value


_WS = {}
WS_ELEMS = 32 << 20  # 128 MiB of f32 split-K slabs per device


def workspace(device, nelem=WS_ELEMS):
    """Persistent f32 scratch (split-K slabs) per device AND stream: stream-ordered reuse only, so kernels on
    the weight-gradient side stream (side_stream) get their own buffer."""
    sid = torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0
    key = (device.type, device.index, sid)
    w = _WS.get(key)
    if w is None or w.numel() < nelem:
        w = torch.empty(nelem, dtype=torch.float32, device=device)
        _WS[key] = w
    return w


# ---------------------------------------------------------------- weight-gradient side stream
# In a backward pass the weight gradient of a layer (dW = X^T dY) and its data gradient (dX = dY W^T) are
# independent: only dX is on the critical path to the earlier layers. With direct arena accumulation the weight
# gradient runs on a second HIP stream, concurrently with the dgrad chain: it fills the tail waves of the dgrad
# GEMMs and the latency-bound BatchNorm reduction launches that otherwise leave CUs idle. The side stream joins the
# main stream before anything reads the gradient arena (bucket all-reduce, optimizer: join_side_streams).
_SIDE = {}
_SIDE_USED = set()
SIDE_STREAM_ON = __import__("os").environ.get("DTF_WGRAD_STREAM", "1") != "0"


def _own_stream(device):
    """A HIP stream created now by the kernel library (dtf_stream_create), not drawn from PyTorch's stream pool."""
    with torch.cuda.device(device):
        h = _native.kernels().dtf_stream_create(0)
    if not h:
        return torch.cuda.Stream(device=device)
    return torch.cuda.ExternalStream(h, device=device)


def side_stream(device):
    s = _SIDE.get(device.index)
    if s is None:
        s = _own_stream(device)
        _SIDE[device.index] = s
    return s


def reserve_streams(device):
    """Create the framework's side stream before anything else creates streams (the process group / RCCL, the
    stream pool): at HIP's default of 4 hardware queues per process the main stream, the side stream and RCCL's
    stream then sit on queues of their own, with no GPU_MAX_HW_QUEUES override."""
    if device.type == "cuda":
        side_stream(device)


# Gradients parked on a ResidualGradLink are overwritten IN PLACE later in the same backward (the first conv / dense
# of the branch accumulates its data gradient into them). A side-stream weight gradient that reads such a tensor
# (GPT-2: the FFN2 / attention-output projection's dW and bias reduce read the block-output gradient) must have run
# before that overwrite: fork_side records an event after those side kernels and ResidualGradLink.take makes the
# overwriting stream wait on it (before_overwrite). Without it the overwrite raced the side reads whenever the side
# stream ran late (P2P bucket kernels waiting on a peer rank there; hipGraph replay).
_PARKED = set()      # storage pointers of parked gradients
_SIDE_READS = {}     # storage pointer -> event on the side stream after the kernels that read it


def _sptr(t):
    return t.untyped_storage().data_ptr()


def mark_parked(t):
    if t is not None and t.is_cuda:
        _PARKED.add(_sptr(t))


def before_overwrite(t):
    """The current stream waits for the side-stream kernels that read `t` (fork_side) before t is overwritten."""
    if t is None or not t.is_cuda:
        return
    p = _sptr(t)
    _PARKED.discard(p)
    ev = _SIDE_READS.pop(p, None)
    if ev is not None:
        if isinstance(ev, tuple):  # a per-stream capture's flag mark (SplitCapture.mark)
            _SPLIT.wait_mark(torch.cuda.current_stream(t.device), ev)
            return
        torch.cuda.current_stream(t.device).wait_event(ev)
        if torch.cuda.is_current_stream_capturing():
            _CAPTURE_KEEP.append(ev)


# Tensors read by side-stream work stay REFERENCED until that work has run. Autograd sums the gradients of a
# tensor with several consumers IN PLACE into the first-arrived gradient when it holds the only reference to its
# storage (torch InputBuffer::accumulate): e.g. a residual add's backward hands the same dy to the branch (whose
# weight gradient reads it on the side stream) and to the shortcut, where the other branch's gradient is then added
# into dy on the main stream. With a second reference held here autograd adds out of place instead. Entries are
# dropped once their event completed (eager; polled at every fork) or when the main stream joins the side stream.
_SIDE_HOLD = []      # (event recorded after the side work, tensors it reads)


_CAPTURE_KEEP = []   # events recorded during a hipGraph capture: destroyed only after the capture ended


def _drop_holds():
    """Forget the held side reads (the main stream is ordered after them now). Inside a capture the events stay
    alive until the capture is over: destroying an event a captured node records crashes the graph's capture end."""
    if _SIDE_HOLD and torch.cuda.is_current_stream_capturing():
        _CAPTURE_KEEP.extend(h[0] for h in _SIDE_HOLD if h[0] is not None)
    elif _CAPTURE_KEEP and not torch.cuda.is_current_stream_capturing():
        _CAPTURE_KEEP.clear()
    _SIDE_HOLD.clear()


def _release_side_holds():
    if not _SIDE_HOLD or torch.cuda.is_current_stream_capturing():
        return
    keep = [h for h in _SIDE_HOLD if h[0] is not None and not h[0].query()]
    _SIDE_HOLD[:] = keep


@contextlib.contextmanager
def fork_side(device, *tensors):
    """Issue side-stream work: the side stream first waits for the main stream's work so far; the tensors it reads
    stay allocated AND referenced until the side stream is done with them (see _SIDE_HOLD), and parked gradients
    among them are protected from their in-place overwrite (before_overwrite)."""
    _release_side_holds()
    side = side_stream(device)
    stream_wait(side, torch.cuda.current_stream(device))
    held = [t for t in tensors if t is not None]
    for t in held:
        t.record_stream(side)
    _SIDE_USED.add(device.index)
    with torch.cuda.stream(side):
        yield side
    parked = [t for t in held if _sptr(t) in _PARKED] if _PARKED else []
    if _SPLIT is not None:
        _SIDE_HOLD.append((None, held))
        if parked:
            mk = _SPLIT.mark(side)
            for t in parked:
                _SIDE_READS[_sptr(t)] = mk
        return
    ev = torch.cuda.Event()
    ev.record(side)
    _SIDE_HOLD.append((ev, held))
    for t in parked:
        _SIDE_READS[_sptr(t)] = ev


def collective_ctx(device):
    """Where a bucket's collective is issued: the weight-gradient side stream, after it waits for the main stream's
    work so far (an event). The bucket's gradients come from both streams; ProcessGroupNCCL then makes its own
    RCCL stream wait on the side stream, so the all-reduce starts once both producers passed this point while the
    dgrad chain keeps running on main. No stream of its own: main + side + RCCL's stream fit HIP's default 4
    hardware queues. (The side stream already waits for main at every weight-gradient fork, so this adds no
    serialisation.) The step joins through the collectives' Work.wait() on the main stream."""
    import contextlib
    if device.type != "cuda":
        return contextlib.nullcontext()
    side = side_stream(device)
    stream_wait(side, torch.cuda.current_stream(device))
    _SIDE_USED.add(device.index)
    return torch.cuda.stream(side)


# Copy stream of the parameter-server push (PSPushBucketer: inbox copies over xGMI during backward); the PS path
# runs no RCCL, so main + side + this stream stay within 4 hardware queues.
_COMM = {}
_COMM_USED = set()


def comm_stream(device):
    s = _COMM.get(device.index)
    if s is None:
        s = _COMM[device.index] = _own_stream(device)
    return s


def comm_stream_ctx(device):
    """Where to issue a PS push copy over arena gradients: the copy stream, waiting on events recorded NOW on the
    main stream and, when weight gradients are in flight there, on the weight-gradient side stream. Neither compute
    stream waits for the copies until the step's join (join_comm_stream)."""
    import contextlib
    if device.type != "cuda":
        return contextlib.nullcontext()
    comm = comm_stream(device)
    stream_wait(comm, torch.cuda.current_stream(device))  # = record an event on main, make comm wait on it
    if device.index in _SIDE_USED:
        stream_wait(comm, _SIDE[device.index])
    _COMM_USED.add(device.index)
    return torch.cuda.stream(comm)


def join_comm_stream(device):
    """The current stream waits for everything issued on the communication stream (a no-op when unused)."""
    if device.type == "cuda" and device.index in _COMM_USED:
        stream_wait(torch.cuda.current_stream(device), _COMM[device.index])
        _COMM_USED.discard(device.index)


_UPD = {}


def update_stream_ctx(device, extra_wait=None):
    """Stream for the per-bucket optimizer updates issued during backward (collective.GradientBucketer with an
    optimizer attached): it waits for the main stream and the weight-gradient side stream as they are now (so
    the bucket's gradients are complete and every kernel that reads the bucket's weights was issued before
    it), and neither of them ever waits for it until the step ends (join_update_stream)."""
    u = _UPD.get(device.index)
    if u is None:
        u = _UPD[device.index] = torch.cuda.Stream(device=device)
    stream_wait(u, torch.cuda.current_stream(device))
    if device.index in _SIDE_USED:
        stream_wait(u, _SIDE[device.index])
    if device.index in _COMM_USED:  # a bucket reduced on the communication stream (P2P / native RCCL)
        stream_wait(u, _COMM[device.index])
    return torch.cuda.stream(u)


def join_update_stream(device):
    u = _UPD.get(device.index)
    if u is not None:
        stream_wait(torch.cuda.current_stream(device), u)


def join_side_streams():
    """Main stream waits for every side-stream weight gradient issued so far."""
    if _SIDE_READS and torch.cuda.is_current_stream_capturing():
        _CAPTURE_KEEP.extend(_SIDE_READS.values())
    _SIDE_READS.clear()
    _PARKED.clear()
    if not _SIDE_USED:
        _drop_holds()
        return
    for idx in list(_SIDE_USED):
        stream_wait(torch.cuda.current_stream(idx), _SIDE[idx])
    _SIDE_USED.clear()
    _drop_holds()  # the main stream is ordered after every side read now


# ---------------------------------------------------------------- per-stream hipGraph capture
# graphs.CapturedStep captures a multi-stream step as one hipGraph PER STREAM (csrc/kernels/graph_sync.hip explains
# why and how the graphs are ordered). While such a capture runs, every cross-stream dependency of the framework goes
# through stream_wait / SplitCapture.mark + wait_mark instead of torch's wait_stream / wait_event, which inside a
# capture would merge the streams into one multi-branch graph.
_SPLIT = None
# A join that waits on a stream holding cross-rank collectives waits as long as a peer may legitimately lag (rank 0
# alone checkpointing or evaluating): the same bound as the P2P all-reduce (parallel/p2p.py). On a timeout the wait
# sets SplitCapture.err; the captured optimizer launch reads that flag and applies nothing (step_abort_ptr), and the
# executor raises at its next per-replay check (graphs.CapturedStep), so a late peer can never make a replica apply
# an unreduced gradient.
XS_TIMEOUT_MS = 300000
_SPLIT_BLOCKERS = __import__("weakref").WeakSet()  # objects whose stream use the per-stream capture cannot express


def block_split_capture(obj):
    """`obj` issues cross-stream work outside the framework's stream helpers (torch.distributed process-group
    collectives: their Work.wait() orders on RCCL's internal stream): hipGraph capture keeps one multi-branch graph
    while it lives."""
    _SPLIT_BLOCKERS.add(obj)


def split_capture_ok():
    return len(_SPLIT_BLOCKERS) == 0


class SplitCapture:
    """State of one per-stream capture: the streams in launch order (main first), each non-main stream's CUDAGraph
    (capture begun lazily at the stream's first use), the external events and the device flag / epoch arrays."""
    MAX_SLOTS = 4096

    def __init__(self, device, pool):
        self.device, self.pool = device, pool
        self.lib = _native.kernels()
        self.streams, self.index, self.graphs = [], {}, []
        self.events = []
        self.nslot = 0
        self.flags = torch.zeros(self.MAX_SLOTS, dtype=torch.int32, device=device)
        self.epochs = torch.zeros(16, dtype=torch.int32, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.counts = {"event": 0, "flag": 0}
        self.activity = {}   # position -> count of waits it took (work is issued on a stream after its waits)
        self.joined = {}     # (consumer, producer) -> producer's activity when consumer last waited for all of it

    def _call(self, name, *args):
        rc = getattr(self.lib, name)(*args)
        if rc:
            raise RuntimeError(f"{name} failed during a per-stream capture: {rc}")

    def begin(self, main):
        """`main` is capturing already (the caller's CUDAGraph); it becomes position 0."""
        self.index[main.cuda_stream] = 0
        self.streams.append(main)
        self.graphs.append(None)
        self._call("dtf_xs_epoch_inc", ptr(self.epochs), 0, main.cuda_stream)

    def ensure(self, s):
        pos = self.index.get(s.cuda_stream)
        if pos is not None:
            return pos
        pos = len(self.streams)
        if pos >= self.epochs.numel():
            raise RuntimeError("per-stream capture: too many streams")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):  # a private memory pool per stream graph (one pool cannot record two captures)
            g.capture_begin(capture_error_mode="relaxed")
        self.index[s.cuda_stream] = pos
        self.streams.append(s)
        self.graphs.append(g)
        self._call("dtf_xs_epoch_inc", ptr(self.epochs), pos, s.cuda_stream)
        return pos

    def _slot(self):
        if self.nslot >= self.MAX_SLOTS:
            raise RuntimeError("per-stream capture: out of flag slots")
        self.nslot += 1
        return self.nslot - 1

    def mark(self, producer):
        """A point on `producer`'s stream that any stream can wait for later (wait_mark)."""
        pp = self.ensure(producer)
        if pp == 0:
            ev = self.lib.dtf_event_create()
            self.events.append(ev)
            self._call("dtf_event_record_external", ev, producer.cuda_stream)
            return ("ev", ev)
        slot = self._slot()
        self._call("dtf_xs_signal", ptr(self.flags), slot, ptr(self.epochs), pp, producer.cuda_stream)
        return ("flag", slot)

    def wait_mark(self, consumer, mk):
        pc = self.ensure(consumer)
        if mk[0] == "ev":
            self.counts["event"] += 1
            self._call("dtf_stream_wait_external", consumer.cuda_stream, mk[1])
        else:
            self.counts["flag"] += 1
            self._call("dtf_xs_wait", ptr(self.flags), mk[1], ptr(self.epochs), pc, ptr(self.err), XS_TIMEOUT_MS,
                       consumer.cuda_stream)

    def wait(self, consumer, producer):
        if consumer.cuda_stream == producer.cuda_stream:
            return
        pp = self.index.get(producer.cuda_stream)
        if pp is None:
            return  # nothing issued on the producer in this capture
        pc = self.ensure(consumer)
        act = self.activity.get(pp, 0)
        if pp > 0 and self.joined.get((pc, pp)) == act:
            return  # the producer took no new work since the consumer last waited for all of it
        self.joined[(pc, pp)] = act
        self.activity[pc] = self.activity.get(pc, 0) + 1
        if pp < pc:  # the producer's graph is enqueued first: an external event pair
            ev = self.lib.dtf_event_create()
            self.events.append(ev)
            self._call("dtf_event_record_external", ev, producer.cuda_stream)
            self.counts["event"] += 1
            self._call("dtf_stream_wait_external", consumer.cuda_stream, ev)
        else:
            self.wait_mark(consumer, self.mark(producer))

    def finish(self):
        """Join every other stream into main (the next replay's main graph must not overwrite buffers a late stream
        still reads) and end their captures."""
        main = self.streams[0]
        for s in self.streams[1:]:
            self.wait(main, s)
        for s, g in zip(self.streams[1:], self.graphs[1:]):
            with torch.cuda.stream(s):
                g.capture_end()
        self.graphs_done = True

    def abort(self):
        for s, g in zip(self.streams[1:], self.graphs[1:]):
            try:
                with torch.cuda.stream(s):
                    g.capture_end()
            except RuntimeError:
                pass

    def replay_others(self):
        """After the main graph was launched on the current stream: every other stream's graph, in order."""
        for s, g in zip(self.streams[1:], self.graphs[1:]):
            with torch.cuda.stream(s):
                g.replay()

    def __del__(self):
        lib = getattr(self, "lib", None)
        for ev in getattr(self, "events", ()):
            try:
                lib.dtf_event_destroy(ev)
            except Exception:
                pass


def step_abort_ptr():
    """Device address of the running per-stream capture's error flag (None outside such a capture): kernels that
    commit a step's result (the fused optimizer) skip their work when it is set."""
    return ptr(_SPLIT.err) if _SPLIT is not None else None


def set_split_capture(sc):
    global _SPLIT
    _SPLIT = sc


def stream_wait(consumer, producer):
    """`consumer` waits for the work issued on `producer` so far (torch's wait_stream, or its per-stream-capture
    form while one runs)."""
    if _SPLIT is not None:
        _SPLIT.wait(consumer, producer)
    else:
        consumer.wait_stream(producer)


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_GET_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


def stream(device=None):
    """Raw handle of the current stream of `device` (default: the current device). Pass the device of the tensors
    a native call touches when it may differ from the current device. (Every kernel launch asks for it: the raw
    accessor skips building a torch.cuda.Stream object — a few microseconds of host time per launch, which adds up
    to milliseconds per training step of a launch-heavy model.)"""
    if _RAW_STREAM is not None and _GET_DEVICE is not None:
        if device is None:
            idx = _GET_DEVICE()
        elif isinstance(device, int):
            idx = device
        else:
            idx = device.index if device.index is not None else _GET_DEVICE()
        return _RAW_STREAM(idx)
    return torch.cuda.current_stream(device).cuda_stream


# ---------------------------------------------------------------- per-step dropout stream
# Dropout kernels hash (host seed, device step counter, element index). An automatically drawn host seed names
# the call site within a step; the device counter names the step and is advanced by `advance_rng` at the start
# of every Model.train_step, as a kernel, so a hipGraph-captured step (whose kernel arguments are frozen at
# capture) still draws a fresh mask on every replay. Explicit user seeds bypass the counter (stateless ops:
# the same seed gives the same mask).
_RNG = {}


def rng_counter(device):
    """Device pointer of the step counter for `device` (created on first use, never inside a capture)."""
    key = (device.type, device.index)
    t = _RNG.get(key)
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("dropout RNG counter first used inside a hipGraph capture: run an eager step first")
        t = torch.zeros(1, dtype=torch.int64, device=device)
        _RNG[key] = t
    return t.data_ptr()


def advance_rng(device):
    """Next training step: new dropout masks everywhere (no-op until a dropout kernel has run on `device`)."""
    t = _RNG.get((device.type, device.index))
    if t is not None and device.type == "cuda":
        call("dtf_rng_advance", t.data_ptr(), stream())


def on_gpu(*ts) -> bool:
    for t in ts:
        if t is not None and isinstance(t, torch.Tensor):
            return t.is_cuda
    return False


def K():
    """The kernel library; raises loudly when it is absent (no silent eager fallback on GPU)."""
    return _native.kernels()


_CALL_LOG = []  # active call_log() counters (tests: which native entry points an op reached)


def call(name, *args):
    fn = getattr(K(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")
    if _CALL_LOG:
        for c in _CALL_LOG:
            c[name] += 1


@contextlib.contextmanager
def call_log():
    """Counts the native entry points called inside the block (collections.Counter by name)."""
    import collections
    c = collections.Counter()
    _CALL_LOG.append(c)
    try:
        yield c
    finally:
        _CALL_LOG.remove(c)


LAUNCH_COUNTERS = ("w4_256", "w4_128", "gemm256", "gemm_tile", "gemm_dact", "beta_bf16", "splitk", "w4f8_256", "w4f8_128",
                   "gemm256_fp8")


def launch_counts():
    """Host-side launch counters of the GEMM dispatch (csrc/kernels/common.h LaunchCounter): which kernel a GEMM
    reached. Take two snapshots and subtract."""
    import ctypes
    n = len(LAUNCH_COUNTERS)
    buf = (ctypes.c_long * n)()
    K().dtf_launch_counts(ctypes.addressof(buf), n)
    return dict(zip(LAUNCH_COUNTERS, list(buf)))


def launch_delta(before):
    after = launch_counts()
    return {k: after[k] - before[k] for k in after}


def contig(t):
    return t if t is None or t.is_contiguous() else t.contiguous()


def bf16_shadow(param):
    """bf16 compute copy of an f32 master variable (kept fresh by the fused optimizer)."""
    s = getattr(param, "_dtf_bf16", None)
    ver = getattr(param, "_dtf_version", None)
    cur = param._version
    if s is None:
        s = param.detach().to(BF16)
        try:
            param._dtf_bf16 = s
        except AttributeError:
            pass
        param._dtf_version = cur
        param._dtf_bf16_owned = True
        return s
    if getattr(param, "_dtf_bf16_owned", False) and ver != cur:
        s.copy_(param.detach())
        param._dtf_version = cur
    return s


class _WeightsEpoch:
    """Bumped by every fused optimizer step: derived weight layouts (e.g. the
    CRSK filter copy used by conv data-gradients) are refreshed lazily."""
    value = 0


def bump_weights_epoch():
    _WeightsEpoch.value += 1


def weights_epoch():
    return _WeightsEpoch.value


_CRSK = []        # weakrefs of the filters that own a CRSK copy
_CRSK_TABLES = {}  # (device, filter set) -> device descriptor table for the batched transform


def _crsk_key(p):
    return (weights_epoch(), p._version)


def crsk_shadow(param, K, RS, C):
    """bf16 [C][R][S][K] copy of a KRSC filter for the dgrad implicit GEMM.

    The copies go stale together (every optimizer step updates every filter), so a miss refreshes ALL stale
    registered filters of the device in one batched launch (dtf_filters_to_crsk: LDS-tiled transposes) rather
    than one launch per conv in the backward pass."""
    import weakref
    s = getattr(param, "_dtf_crsk", None)
    if s is not None and getattr(param, "_dtf_crsk_key", None) == _crsk_key(param):
        return s
    if s is None:
        s = torch.empty((C, RS, K), dtype=BF16, device=param.device)
        param._dtf_crsk = s
        param._dtf_crsk_geom = (K, RS, C)
        _CRSK.append(weakref.ref(param))
    live = []
    for r in list(_CRSK):
        p = r()
        if p is None:
            _CRSK.remove(r)
            continue
        if p.device == param.device and getattr(p, "_dtf_crsk_key", None) != _crsk_key(p):
            live.append(p)
    if not any(p is param for p in live):
        live.append(param)
    if len(live) == 1:
        call("dtf_filter_to_crsk", ptr(bf16_shadow(param)), ptr(s), K, RS, C, stream())
    else:
        rows, tiles = [], 0
        for p in live:
            k, rs, c = p._dtf_crsk_geom
            rows.append((ptr(bf16_shadow(p)), ptr(p._dtf_crsk), k, rs, c, tiles))
            tiles += rs * ((k + 63) // 64) * ((c + 63) // 64)
        tkey = (param.device.index, tuple(rows))
        table = _CRSK_TABLES.get(tkey)
        if table is None and torch.cuda.is_current_stream_capturing():
            # a filter set first seen inside a hipGraph capture (no host->device copy allowed): one launch each
            for p in live:
                k, rs, c = p._dtf_crsk_geom
                call("dtf_filter_to_crsk", ptr(bf16_shadow(p)), ptr(p._dtf_crsk), k, rs, c, stream())
        else:
            if table is None:
                if len(_CRSK_TABLES) > 64:
                    _CRSK_TABLES.clear()
                table = torch.tensor(rows, dtype=torch.int64).to(param.device)
                _CRSK_TABLES[tkey] = table
            call("dtf_filters_to_crsk", ptr(table), len(rows), tiles, stream())
    for p in live:
        p._dtf_crsk_key = _crsk_key(p)
    return s


# ---------------------------------------------------------------- direct gradient accumulation
# Inside Model.train_step's backward the parameters' .grad are views of the flat arena gradient, zeroed by
# the fused optimizer every step. Ops with hand-written backwards may then accumulate a parameter's gradient
# straight into that view (GEMM beta=1 / accumulate flags) and return None to autograd, which saves one
# AccumulateGrad add kernel + one temporary per parameter. Autograd still visits the parameter's
# AccumulateGrad node (with an undefined gradient), so post-accumulate hooks (gradient bucketing) fire
# unchanged. Outside `direct_grads()` (GradientTape, custom loops) every op returns its grads.
_direct = [False]


class direct_grads:
    def __enter__(self):
        self._prev = _direct[0]
        _direct[0] = True
        return self

    def __exit__(self, *exc):
        _direct[0] = self._prev


def direct_grad(p):
    """The arena gradient view to accumulate p's gradient into, or None (return the gradient instead)."""
    if not _direct[0] or p is None or not getattr(p, "requires_grad", False):
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.shape != p.shape:
        return None
    return g if g.data_ptr() == getattr(p, "_dtf_grad_ptr", -1) else None
