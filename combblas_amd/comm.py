"""Collectives of the distributed SpGEMM drivers, over torch.distributed.

On MI355X the process group is "nccl" (= RCCL over xGMI) and every collective runs directly on
HBM tensors. With the "gloo" backend (CPU multi-process tests, or several ranks sharing one GPU
on a test box) device tensors are staged through host memory, because gloo implements only a
subset of its collectives for device tensors.

The reference's MPI calls each helper replaces:
  bcast      MPI_Bcast of the Dcsc arrays            SpParHelper::BCastMatrix, SpParHelper.cpp:581-599
  ibcast     MPI_Ibcast of the Dcsc arrays           SpParHelper::IBCastMatrix (Mult_AnXBn_Overlap,
                                                     ParFriends.h:1150-1200)
  allgather  MPI_Allgather of the 4 essentials        SpParHelper::GetSetSizes, SpParHelper.cpp:797-808
  alltoallv  MPI_Alltoall(profile) + MPI_Alltoallv    Mult_AnXBn_SUMMA3D, ParFriends.h:3137-3160
  allreduce  MPI_Allreduce                            (phase planning, statistics)
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class Group:
    """A communicator: an ordered list of global ranks plus its torch.distributed group.

    `groups()` must be created collectively (every rank calls Group(...) for every group in the
    same order, as MPI_Comm_split requires every rank of the parent)."""

    def __init__(self, ranks, me):
        self.ranks = list(ranks)
        self.size = len(self.ranks)
        self.rank = self.ranks.index(me) if me in self.ranks else -1
        self.pg = None
        if dist.is_initialized() and dist.get_world_size() > 1:
            pg = dist.new_group(self.ranks)
            self.pg = pg if self.rank >= 0 else None

    def global_rank(self, r):
        return self.ranks[r]


def _staged(t: torch.Tensor) -> bool:
    return t.is_cuda and dist.get_backend() == "gloo"


def bcast(t: torch.Tensor, root: int, g: Group) -> torch.Tensor:
    """In-place broadcast of `t` from group rank `root` (a no-op for a one-rank group)."""
    if g.size == 1 or t.numel() == 0:
        return t
    src = g.global_rank(root)
    if _staged(t):
        h = t.cpu()
        dist.broadcast(h, src=src, group=g.pg)
        if g.rank != root:
            t.copy_(h)
        return t
    dist.broadcast(t, src=src, group=g.pg)
    return t


class _Done:
    def wait(self):
        return None


class _StagedBcast:
    """an async broadcast of a host copy; wait() lands it in the device tensor"""

    def __init__(self, work, h, t, copy):
        self.work, self.h, self.t, self.copy = work, h, t, copy

    def wait(self):
        self.work.wait()
        if self.copy:
            self.t.copy_(self.h)


def ibcast(t: torch.Tensor, root: int, g: Group):
    """Non-blocking broadcast of `t` from group rank `root`; returns a request with wait().

    With RCCL the copy runs on the communicator's stream while the caller's stream keeps
    computing; wait() makes the caller's current stream wait for it (no host sync)."""
    if g.size == 1 or t.numel() == 0:
        return _Done()
    src = g.global_rank(root)
    if _staged(t):
        h = t.cpu() if g.rank == root else torch.empty(t.shape, dtype=t.dtype)
        return _StagedBcast(dist.broadcast(h, src=src, group=g.pg, async_op=True), h, t, g.rank != root)
    return dist.broadcast(t, src=src, group=g.pg, async_op=True)


def allgather_i64(vals, g: Group, device) -> torch.Tensor:
    """Every rank's int64 vector (same length everywhere) -> [g.size, len] (host tensor)."""
    x = torch.tensor(list(vals), dtype=torch.int64, device=device)
    if g.size == 1:
        return x.view(1, -1).cpu()
    if dist.get_backend() == "gloo":
        x = x.cpu()
    out = [torch.empty_like(x) for _ in range(g.size)]
    dist.all_gather(out, x, group=g.pg)
    return torch.stack([o.cpu() for o in out])


def allreduce_(t: torch.Tensor, g: Group, op=dist.ReduceOp.SUM) -> torch.Tensor:
    if g.size == 1:
        return t
    if _staged(t):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=g.pg)
        t.copy_(h)
        return t
    dist.all_reduce(t, op=op, group=g.pg)
    return t


def alltoallv(send: torch.Tensor, send_counts, recv_counts, g: Group) -> torch.Tensor:
    """Personalised exchange of a 1-D tensor: send[s_off[j]:s_off[j]+send_counts[j]] goes to group
    rank j; returns the concatenation of what every rank sent here, in group-rank order."""
    send_counts = [int(c) for c in send_counts]
    recv_counts = [int(c) for c in recv_counts]
    if g.size == 1:
        return send[: send_counts[0]].clone()
    out = torch.empty(sum(recv_counts), dtype=send.dtype, device=send.device)
    if sum(send_counts) == 0 and sum(recv_counts) == 0:
        return out
    if dist.get_backend() == "gloo":
        # gloo has no alltoallv for device tensors; stage and express it as per-peer broadcasts
        # of the host buffer (test path only; RCCL's alltoall is used on MI355X)
        hs = send.cpu()
        ho = torch.empty(sum(recv_counts), dtype=send.dtype)
        s_off = [0]
        for c in send_counts:
            s_off.append(s_off[-1] + c)
        r_off = [0]
        for c in recv_counts:
            r_off.append(r_off[-1] + c)
        reqs = []
        for j in range(g.size):
            if j == g.rank:
                ho[r_off[j]:r_off[j + 1]] = hs[s_off[j]:s_off[j + 1]]
                continue
            if send_counts[j]:
                reqs.append(dist.isend(hs[s_off[j]:s_off[j + 1]].contiguous(), dst=g.global_rank(j), group=g.pg))
            if recv_counts[j]:
                reqs.append(dist.irecv(ho[r_off[j]:r_off[j + 1]], src=g.global_rank(j), group=g.pg))
        for r in reqs:
            r.wait()
        out.copy_(ho)
        return out
    dist.all_to_all_single(out, send.contiguous(), output_split_sizes=recv_counts, input_split_sizes=send_counts,
                           group=g.pg)
    return out
