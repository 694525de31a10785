"""Collective helpers of the GPU data plane (RCCL over xGMI; gloo on CPU for tests).

The PS message patterns map onto collectives:
  C1/C2 sparse Get      -> all-to-all(counts) + all-to-all-v(keys) + all-to-all-v(rows)
  C3    sparse Add      -> all-to-all-v(grad rows) into the owner shards
  C1/C3 dense Get/Add   -> reduce-scatter(grads) / all-gather(params) of equal shards
  C6    Barrier         -> 1-element all-reduce on the group
With one rank every collective degenerates to a local copy (no RCCL launch at all).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class CommStats:
    bytes_a2a: int = 0
    bytes_rs: int = 0
    bytes_ag: int = 0
    calls: int = 0

    def as_dict(self):
        return dict(bytes_a2a=self.bytes_a2a, bytes_rs=self.bytes_rs, bytes_ag=self.bytes_ag, calls=self.calls)


class Comm:
    """Rank/world/device bookkeeping plus the collectives used by the tables."""

    def __init__(self, group=None, device: torch.device | None = None):
        self.initialized = dist.is_available() and dist.is_initialized()
        self.group = group
        self.rank = dist.get_rank(group) if self.initialized else 0
        self.world = dist.get_world_size(group) if self.initialized else 1
        self.backend = dist.get_backend(group) if self.initialized else "none"
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        self.device = device
        self.stats = CommStats()
        self._lanes: dict[str, Comm] = {}
        self._plan_stream = None

    def lane(self, name: str) -> "Comm":
        """A named extra communicator over the same ranks, for collectives issued on their own HIP
        stream (key planning, sparse push, dense clock): ops of ONE communicator are serialised
        in issue order, so work that must overlap needs separate communicators, which progress
        independently. Creating one is collective (first call on every rank, in the same order
        -- the tables do it in their constructors)."""
        if self.world == 1:
            return self
        if name not in self._lanes:
            ranks = list(range(self.world)) if self.group is None else dist.get_process_group_ranks(self.group)
            c = Comm(group=dist.new_group(ranks), device=self.device)
            c.stats = self.stats  # one byte account per rank
            self._lanes[name] = c
        return self._lanes[name]

    def background(self) -> "Comm":
        """The side-stream communicator of SSP/ASP clock work (see lane())."""
        return self.lane("bg")

    def plan_stream(self):
        """The HIP stream on which lookahead key planning runs (one per rank, shared by tables)."""
        if self._plan_stream is None and self.device.type == "cuda":
            self._plan_stream = torch.cuda.Stream(device=self.device)
        return self._plan_stream

    # -- helpers ------------------------------------------------------------------------
    def _staged(self, *ts) -> bool:
        """GPU tensors over a gloo group: the multi-rank GPU TEST harness (several ranks sharing
        one card, where RCCL refuses duplicate devices) stages them through host memory, so the
        streams / lanes / lookahead logic runs on the GPU at world > 1. Never a production path:
        init_distributed() picks RCCL whenever GPUs are present."""
        return self.backend == "gloo" and any(t.is_cuda for t in ts)

    @staticmethod
    def _host(t: torch.Tensor) -> torch.Tensor:
        # gloo moves raw 16-bit payloads as fp16 bit patterns (it has no bf16 / int16 path)
        t = t.detach().cpu()
        return t.view(torch.float16) if t.dtype == torch.bfloat16 else t

    @staticmethod
    def _back(dst: torch.Tensor, host: torch.Tensor):
        dst.copy_(host.view(dst.dtype) if dst.dtype == torch.bfloat16 else host)

    def all_to_all_v(self, out: torch.Tensor, inp: torch.Tensor, recv_splits: list[int], send_splits: list[int],
                     p2p: bool = False):
        """Rows of ``inp`` split by ``send_splits`` go to ranks 0..P-1; ``out`` gets recv_splits.

        p2p=True issues the exchange as grouped point-to-point send/recv pairs (one per peer
        with a non-empty message, the own segment copied locally) -- the SSP/ASP data path;
        otherwise one RCCL all-to-all-v."""
        if self.world > 1 and self._staged(out, inp):
            o = self._host(out[: sum(recv_splits)])
            self.all_to_all_v(o, self._host(inp[: sum(send_splits)]), recv_splits, send_splits, p2p)
            self._back(out[: sum(recv_splits)], o)
            return out
        self.stats.calls += 1
        if self.world == 1:
            n = send_splits[0]
            if n:
                out[:n].copy_(inp[:n])
            return out
        self.stats.bytes_a2a += inp[: sum(send_splits)].numel() * inp.element_size()
        if not p2p:
            o = out[: sum(recv_splits)]
            i = inp[: sum(send_splits)]
            dist.all_to_all_single(o, i, recv_splits, send_splits, group=self.group)
            return out
        so = [0]
        for c in send_splits:
            so.append(so[-1] + c)
        ro = [0]
        for c in recv_splits:
            ro.append(ro[-1] + c)
        ops_ = []
        for peer in range(self.world):
            if peer == self.rank:
                if send_splits[peer]:
                    out[ro[peer]: ro[peer + 1]].copy_(inp[so[peer]: so[peer + 1]])
                continue
            if send_splits[peer]:
                ops_.append(dist.P2POp(dist.isend, inp[so[peer]: so[peer + 1]].contiguous(), peer, group=self.group))
            if recv_splits[peer]:
                ops_.append(dist.P2POp(dist.irecv, out[ro[peer]: ro[peer + 1]], peer, group=self.group))
        if ops_:
            for r in dist.batch_isend_irecv(ops_):
                r.wait()
        return out

    def all_to_all_counts(self, recv: torch.Tensor, counts: torch.Tensor):
        """Device-side all-to-all of per-destination counts (no host sync)."""
        if self.world == 1:
            recv.copy_(counts)
        elif self._staged(recv, counts):
            r = torch.empty(recv.shape, dtype=recv.dtype)
            dist.all_to_all_single(r, counts.cpu(), group=self.group)
            recv.copy_(r)
        else:
            dist.all_to_all_single(recv, counts, group=self.group)
        return recv

    def exchange_counts(self, counts: torch.Tensor) -> tuple[list[int], list[int]]:
        """all-to-all of per-destination counts; returns (send, recv) as host lists (1 sync)."""
        if self.world == 1:
            c = counts.tolist()
            return c, c
        recv = torch.empty_like(counts)
        self.all_to_all_counts(recv, counts)
        both = torch.stack([counts, recv]).cpu()
        return both[0].tolist(), both[1].tolist()

    def reduce_scatter(self, out_shard: torch.Tensor, inp: torch.Tensor):
        if self.world > 1 and self._staged(out_shard, inp):
            o = torch.empty(out_shard.shape, dtype=out_shard.dtype)
            self.reduce_scatter(o, inp.cpu())
            out_shard.copy_(o)
            return out_shard
        self.stats.calls += 1
        if self.world == 1:
            out_shard.copy_(inp)
            return out_shard
        self.stats.bytes_rs += inp.numel() * inp.element_size()
        dist.reduce_scatter_tensor(out_shard, inp, group=self.group)
        return out_shard

    def all_gather(self, out_full: torch.Tensor, shard: torch.Tensor):
        if self.world > 1 and self._staged(out_full, shard):
            o = self._host(out_full)
            self.all_gather(o, self._host(shard).clone())
            self._back(out_full, o)
            return out_full
        self.stats.calls += 1
        if self.world == 1:
            if out_full.data_ptr() != shard.data_ptr():
                out_full.copy_(shard)
            return out_full
        self.stats.bytes_ag += out_full.numel() * out_full.element_size()
        if self.backend == "gloo" and shard.data_ptr() >= out_full.data_ptr() and \
                shard.data_ptr() < out_full.data_ptr() + out_full.numel() * out_full.element_size():
            shard = shard.clone()  # gloo does not support the in-place (aliased) form
        dist.all_gather_into_tensor(out_full, shard, group=self.group)
        return out_full

    def all_reduce_(self, t: torch.Tensor, op=None):
        if self.world == 1:
            return t
        if self._staged(t):
            h = t.cpu()
            dist.all_reduce(h, op=op or dist.ReduceOp.SUM, group=self.group)
            t.copy_(h)
            return t
        dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=self.group)
        return t

    def barrier(self):
        if self.world == 1:
            return
        t = torch.zeros(1, device=self.device)
        self.all_reduce_(t)
        if t.is_cuda:
            torch.cuda.synchronize(self.device)


def init_distributed(backend: str | None = None) -> Comm:
    """Initialise torch.distributed from the torchrun env (RANK/WORLD_SIZE/MASTER_*).

    One process per GPU: the local rank selects the device; backend "nccl" is RCCL on ROCm.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            # MINIPS_DIST_BACKEND=gloo (+ MINIPS_SHARE_DEVICE=1): the multi-rank test harness on one
            # card (RCCL refuses two ranks on one device); production picks RCCL whenever GPUs exist
            backend = os.environ.get("MINIPS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # test harness only: several ranks on one card (MINIPS_SHARE_DEVICE=1 -> all on device 0)
        if os.environ.get("MINIPS_SHARE_DEVICE") == "1":
            local = 0
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
            if torch.cuda.is_available():
                torch.cuda.set_device(local)
    elif torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    return Comm()
