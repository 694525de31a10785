"""Building blocks shared by the dense-tower models on the GPU parameter server.

ParamLayout   names -> (offset, shape) views into one flat parameter vector (the DenseTable
              master / pulled copy / gradient buffer all share the layout).
Linear        bias folded into the weight: W_ext [n_out, k_pad] with the bias in column k_in;
              activations carry a constant-1 column at k_in (see ext_activation), so the
              forward GEMM adds the bias and the weight-gradient GEMM yields the bias gradient.
"""
from __future__ import annotations


import math

import torch

from .. import ops
from ..utils import streams


def align(n: int, a: int = 8) -> int:
    return (n + a - 1) // a * a


class ParamLayout:
    def __init__(self):
        self.entries: dict[str, tuple[int, tuple]] = {}
        self.size = 0

    def add(self, name: str, shape: tuple) -> str:
        n = 1
        for s in shape:
            n *= s
        self.entries[name] = (self.size, tuple(shape))
        self.size += align(n, 64)  # 128-byte aligned segments (bf16 and fp32 views stay 16-B aligned)
        return name

    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        off, shape = self.entries[name]
        n = 1
        for s in shape:
            n *= s
        return buf[off: off + n].view(shape)


def ext_activation(rows: int, k_in: int, device, dtype=torch.bfloat16) -> torch.Tensor:
    """[rows, align8(k_in + 1)] activation buffer whose column k_in is the constant 1."""
    t = torch.zeros(rows, align(k_in + 1), dtype=dtype, device=device)
    t[:, k_in] = 1.0
    return t


class Linear:
    """A bias-folded Linear(k_in -> n_out) living in a ParamLayout."""

    def __init__(self, layout: ParamLayout, name: str, k_in: int, n_out: int, n_pad: int | None = None):
        self.name, self.k_in, self.n_out = name, k_in, n_out
        self.k_pad = align(k_in + 1)
        self.n_rows = n_pad or n_out  # rows beyond n_out stay zero (K-padding of the next dgrad)
        layout.add(name, (self.n_rows, self.k_pad))
        self.layout = layout

    def init(self, full: torch.Tensor, gen, std: float | None = None):
        w = self.layout.view(full, self.name)
        w.zero_()
        if std is None:
            bound = 1.0 / math.sqrt(self.k_in)
            w[: self.n_out, : self.k_in].uniform_(-bound, bound, generator=gen)
        else:
            w[: self.n_out, : self.k_in].normal_(0.0, std, generator=gen)

    def W(self, P):
        return self.layout.view(P, self.name)

    def forward(self, P, x_ext, out, act="relu", aux=None):
        """out[:, :n_out] = act(x_ext W_ext^T); x_ext carries the ones column."""
        W = self.W(P)
        M = x_ext.shape[0]
        if act == "gelu_daux":  # aux <- gelu'(u): the backward multiplies (dgrad gelu_d=aux)
            return ops.gemm(x_ext, W, out, M, self.n_out, self.k_pad, False, False, ops.EPI_BIAS_GELU_DAUX_BF16,
                            mask=aux)
        if act == "gelu_aux":
            return ops.gemm(x_ext, W, out, M, self.n_out, self.k_pad, False, False, ops.EPI_BIAS_GELU_AUX_BF16,
                            mask=aux)
        epi = {"relu": ops.EPI_BIAS_RELU_BF16, "none": ops.EPI_BIAS_BF16}[act]
        return ops.gemm(x_ext, W, out, M, self.n_out, self.k_pad, False, False, epi)

    def wgrad(self, G, dy, x_ext, sink=None):
        """G_W += dy^T x_ext (split-K gemm.hip; the bias gradient lands in column k_in). ``sink``: a
        DenseTable.slab_sink() -- the K slices stay in planes its Adam folds (no reduce kernel)."""
        return ops.linear_wgrad(dy, x_ext, self.W(G), defer=sink)

    def dgrad(self, P, dy, out, mask=None, gelu_u=None, out_f32=False, k_rows=None, gelu_d=None):
        """out = dy W[:, :k_in] (ReLU-masked by `mask`, or times gelu'(gelu_u)).

        The [K][N] weight layout is read 8 columns at a time, so an unaligned k_in computes
        align8(k_in) columns: the extra ones (bias column, zero padding) land in out's padding."""
        W = self.W(P)
        M = dy.shape[0]
        K = k_rows or self.n_rows
        N = align(self.k_in)
        assert out.shape[1] >= N, f"dgrad output needs {N} columns"
        if out_f32:
            return ops.gemm(dy, W, out, M, N, K, False, True, ops.EPI_STORE_F32)
        if gelu_d is not None:  # times the saved derivative gelu'(u)
            return ops.gemm(dy, W, out, M, N, K, False, True, ops.EPI_MUL_AUX_BF16, mask=gelu_d)
        if gelu_u is not None:
            return ops.gemm(dy, W, out, M, N, K, False, True, ops.EPI_GELU_GRAD_BF16, mask=gelu_u)
        if mask is not None:
            return ops.gemm(dy, W, out, M, N, K, False, True, ops.EPI_RELU_MASK_BF16, mask=mask)
        return ops.gemm(dy, W, out, M, N, K, False, True, ops.EPI_STORE_BF16)


def compute_priority() -> int:
    """HIP stream priority for the training step's compute streams (main and weight-gradient side
    stream). High priority (-1), which makes the dispatcher favour their workgroups over the
    planning / data stream's, measured neutral on the W&D step (0.520-0.524 vs 0.519-0.521 ms)
    and worse on GPT-2 (profiles/r4/ab_gpt2_knobs.txt), so normal priority."""
    return 0


def _prev_raw(prev) -> int:
    """Raw handle of the stream saved by streams._get (stream_id, device_index, device_type)."""
    return torch.cuda.Stream(stream_id=prev[0], device_index=prev[1], device_type=prev[2]).cuda_stream


class _Fork:
    """SideStream.fork()'s context: the side stream waits for the current stream, then the block
    runs on the side stream (GEMM splits in overlap mode)."""

    __slots__ = ("side", "prev", "mode", "after")

    def __init__(self, side, after=None):
        self.side = side
        self.after = after

    def __enter__(self):
        sd = self.side
        st = sd.stream
        if st is None:
            return None
        idx = st.device_index
        rec = ops._REC
        if self.after is not None:  # an earlier point of the current stream (SideStream.point)
            if sd._fast:
                self.after.wait(sd._raw)
            else:
                st.wait_event(self.after)
        elif rec is not None:  # recorded into a LaunchList: its own event orders the two streams
            rec.lst.fork(streams.current_raw(idx), sd._raw)
        elif sd._fast:
            ev = sd._event()
            ev.record(streams.current_raw(idx))
            ev.wait(sd._raw)
        else:
            ev = sd._event()
            ev.record(streams.current(idx))
            st.wait_event(ev)
        self.mode = ops.overlap_mode(True)  # forked work: GEMM splits chosen for throughput, not latency
        self.prev = streams._get(idx)
        streams._set(stream_id=st.stream_id, device_index=idx, device_type=st.device_type)
        if streams.DELAY_US > 0:
            if "fork" in streams.DELAY_WHERE:  # the forked work starts late
                streams.delay(sd._raw, idx)
            if "main" in streams.DELAY_WHERE:  # the stream forked FROM continues late
                streams.delay(_prev_raw(self.prev), idx)
        return st

    def __exit__(self, *exc):
        if self.side.stream is None:
            return False
        p = self.prev
        streams._set(stream_id=p[0], device_index=p[1], device_type=p[2])
        ops.overlap_mode(self.mode)
        return False


class SideStream:
    """Fork-join helper: independent work (weight gradients) issued on a second HIP stream.

    ``with side.fork():`` makes the side stream wait for everything issued so far on the current
    stream, then runs the block on the side stream; ``join()`` makes the current stream wait for
    all forked work. Disabled (or on CPU) it is a no-op and the block runs inline. Stream changes
    go through utils/streams (no per-call device resolution: this is the step's hottest host path)."""

    def __init__(self, device, enabled: bool = True, priority: int | None = None):
        """``priority`` (HIP: -1 high, 0 normal, 1 low; default compute_priority()). A low-priority
        weight-gradient stream (the dispatcher then favours the compute stream's workgroups) measured
        within noise on the W&D step (0.3431-0.3479 vs 0.3449-0.3493 ms, profiles/r6/ab_wd_r6.txt)."""
        cuda = enabled and torch.device(device).type == "cuda"
        if priority is None:
            priority = compute_priority()
        if cuda and priority > 0:
            from ..ps.comm import dedicated_stream

            self.stream = dedicated_stream(device, priority)
        else:
            self.stream = torch.cuda.Stream(device=device, priority=priority) if cuda else None
        # fork / join events are re-recorded every step (a wait binds to the record issued before
        # it): no event objects created and destroyed per fork. Same-device ordering only, so
        # fence-free native events (ops_py FastEvent; MINIPS_STREAM_DEBUG sysfence=side: torch events)
        self._fast = self.stream is not None and streams.fast_for("side")
        if self._fast:
            from .._native import kernels

            self._evs = [kernels().FastEvent() for _ in range(8)]
        else:
            self._evs = [torch.cuda.Event() for _ in range(8)] if self.stream is not None else []
        self._raw = self.stream.cuda_stream if self.stream is not None else 0
        self._ev_i = 0

    def _event(self):
        ev = self._evs[self._ev_i % len(self._evs)]
        self._ev_i += 1
        return ev

    def fork(self, after=None):
        """``after``: an event of the current stream from point() -- the side stream waits for the
        current stream only up to that point (work issued since then may overlap the block)."""
        return _Fork(self, after)

    def point(self):
        """An event at the current stream's position now (for fork(after=...)); None when disabled."""
        if self.stream is None:
            return None
        ev = self._event()
        if self._fast:
            ev.record(streams.current_raw(self.stream.device_index))
        else:
            ev.record(streams.current(self.stream.device_index))
        return ev

    def join(self):
        if self.stream is not None:
            idx = self.stream.device_index
            if ops._REC is not None:
                ops._REC.lst.fork(self._raw, streams.current_raw(idx))
                return
            ev = self._event()
            if self._fast:
                ev.record(self._raw)
                ev.wait(streams.current_raw(idx))
            else:
                ev.record(self.stream)
                streams.current(idx).wait_event(ev)

    def mark(self):
        """Event after the work forked so far (None when disabled), from a ring of 16 (every caller
        issues its wait within a few marks); torch-compatible (streams.FastEvent duck-types it)."""
        if self.stream is None:
            return None
        ring = self.__dict__.get("_marks")
        if ring is None:
            ring = self._marks = streams.EventRing(16, fast=self._fast)
        ev = ring.next()
        ev.record(self.stream)
        return ev

    def wait(self, ev):
        """The current stream waits for ``ev`` (before it overwrites a buffer forked work reads)."""
        if ev is None:
            return
        idx = self.stream.device_index
        if isinstance(ev, torch.cuda.Event):
            streams.current(idx).wait_event(ev)
        else:  # ops_py FastEvent or streams.FastEvent
            getattr(ev, "ev", ev).wait(streams.current_raw(idx))


class Replayer:
    """Record-once, replay-after launch sequences of a step (ops.recording into a native
    LaunchList, csrc/bindings/ops_py.cpp). ``replayer(key, fn)``: the first call with ``key`` runs
    ``fn`` -- GEMM-family ops and SideStream forks only -- recording it; later calls replay the
    recorded launches on the current and side streams and repeat the slab-sink registrations. The
    key must name every buffer ``fn`` addresses (a list holds its tensors, so a recorded address
    is never handed to another buffer while the list lives)."""

    def __init__(self, side: SideStream, cap: int = 8):
        self.side = side
        self.cap = cap
        self._lists: dict = {}

    def __call__(self, key, fn):
        idx = self.side.stream.device_index
        main = streams.current_raw(idx)
        e = self._lists.get(key)
        if e is None:
            from .._native import kernels

            if len(self._lists) >= self.cap:
                self._lists.clear()
            lst = kernels().LaunchList(main, self.side._raw)
            with ops.recording(lst) as rec:
                fn()
            self._lists[key] = (lst, rec.sink_adds)
            return
        lst, adds = e
        lst.run(main, self.side._raw)
        for sink, dw, slab, nsplit in adds:
            sink.add(dw, slab, nsplit)
