"""Process-group helpers: one rank per GPU, ``torch.distributed`` over RCCL (``nccl`` backend on ROCm)
or ``gloo`` on the host.

Replaces the reference's Spark ``treeAggregate``/``reduce``/``fold``/``collect`` reductions and XGBoost's
Rabit allreduce. Statistics of one fit stage are packed into a single
flat buffer and reduced in one collective (``bucketed_all_reduce``): the payloads are small and
latency-bound on xGMI, so one call per stage beats one call per statistic.
"""
from __future__ import annotations

import os
from typing import List, Sequence

import torch
import torch.distributed as dist


# Projection mode (scripts/project_schedule.py): one process plays rank `rank` of `world` ranks that all hold
# shards identical to its own -- every collective returns what it would return then (sums scale by the world,
# gathers tile), without any communication. The per-rank share of a multi-GPU run can so be timed on one GPU;
# it is a timing device only (the data of the other ranks is not the real data).
_SIM = None


def simulate(rank_: int, world_: int) -> None:
    global _SIM
    _SIM = (int(rank_), int(world_)) if world_ > 1 else None


def simulated() -> bool:
    return _SIM is not None


def is_dist() -> bool:
    return _SIM is not None or (dist.is_available() and dist.is_initialized())


def rank() -> int:
    if _SIM is not None:
        return _SIM[0]
    return dist.get_rank() if is_dist() else 0


def world() -> int:
    if _SIM is not None:
        return _SIM[1]
    return dist.get_world_size() if is_dist() else 1


def barrier():
    if _SIM is not None:
        return
    if is_dist():
        dist.barrier()


def init_from_env(backend: str = None, device_id: int = None):
    """Initialize from torchrun env vars (RANK, WORLD_SIZE, MASTER_ADDR/PORT); no-op when single-process."""
    if is_dist():
        return
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl" and device_id is not None:
        kw["device_id"] = torch.device("cuda", device_id)
    dist.init_process_group(backend=backend, **kw)


def _comm_device(t: torch.Tensor):
    if _SIM is None and is_dist() and dist.get_backend() == "nccl" and t.device.type != "cuda":
        return torch.device("cuda", torch.cuda.current_device())
    return t.device


class RankGroup:
    """A subset of the ranks that runs collectives of its own: ``ranks`` (global ranks, ascending), this
    process's ``rank`` inside it and the ``torch.distributed`` group (None in projection mode)."""

    def __init__(self, ranks: Sequence[int], pg=None, cpu_pg=None):
        self.ranks = tuple(int(r) for r in ranks)
        self.pg = pg
        self.cpu_pg = cpu_pg        # gloo twin for host-memory collectives when the main backend is nccl
        me = rank()
        self.rank = self.ranks.index(me) if me in self.ranks else -1
        self.world = len(self.ranks)

    @property
    def leader(self) -> int:
        return self.ranks[0]


_PARTITIONS: dict = {}


def partition(group_size: int) -> RankGroup:
    """The group of ``group_size`` consecutive ranks this rank belongs to, out of ``world / group_size``
    groups. Creating process groups is collective over ALL ranks (every rank creates every group, in the
    same order), so every rank must call this at the same point; results are cached per size."""
    n = world()
    if group_size <= 0 or n % group_size != 0:
        raise ValueError(f"group size {group_size} does not divide the world {n}")
    if group_size in _PARTITIONS:
        return _PARTITIONS[group_size]
    me = rank()
    mine = None
    for g in range(n // group_size):
        ranks_g = list(range(g * group_size, (g + 1) * group_size))
        pg = cpu = None
        if _SIM is None and is_dist() and group_size < n:
            pg = dist.new_group(ranks=ranks_g)
            if dist.get_backend() != "gloo":
                cpu = dist.new_group(ranks=ranks_g, backend="gloo")
        elif _SIM is None and is_dist():
            pg = dist.group.WORLD
        if me in ranks_g:
            mine = RankGroup(ranks_g, pg, cpu)
    _PARTITIONS[group_size] = mine
    return mine


def _pg(group):
    return group.pg if isinstance(group, RankGroup) else group


def _gsize(group) -> int:
    if isinstance(group, RankGroup):
        return group.world
    return world()


def all_reduce(t: torch.Tensor, op: str = "sum", group=None) -> torch.Tensor:
    if _SIM is not None:
        return t * _gsize(group) if op == "sum" else t.clone()
    if not is_dist() or _gsize(group) <= 1:
        return t
    dev = _comm_device(t)
    x = t.to(dev)
    o = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
    dist.all_reduce(x, op=o, group=_pg(group))
    return x.to(t.device)


def bucketed_all_reduce(tensors: Sequence[torch.Tensor], op: str = "sum", group=None) -> List[torch.Tensor]:
    """Flatten, reduce once, unflatten (same dtype required per bucket; mixed dtypes go via float64)."""
    if not is_dist() or not tensors:
        return list(tensors)
    dt = torch.float64
    flat = torch.cat([t.reshape(-1).to(dt) for t in tensors])
    flat = all_reduce(flat, op, group)
    out, off = [], 0
    for t in tensors:
        n = t.numel()
        out.append(flat[off:off + n].reshape(t.shape).to(t.dtype))
        off += n
    return out


def all_gather_object(obj) -> list:
    if _SIM is not None:
        import copy
        return [obj] + [copy.deepcopy(obj) for _ in range(_SIM[1] - 1)]
    if not is_dist():
        return [obj]
    out = [None] * world()
    dist.all_gather_object(out, obj)
    return out


def broadcast_object(obj, src: int = 0, group=None):
    """``src`` is a global rank (the group's leader for a :class:`RankGroup`)."""
    if _SIM is not None or not is_dist() or _gsize(group) <= 1:
        return obj
    box = [obj]
    pg = group.cpu_pg or group.pg if isinstance(group, RankGroup) else group
    dist.broadcast_object_list(box, src=src, group=pg)
    return box[0]


def all_gather_rows(t: torch.Tensor) -> torch.Tensor:
    """Concatenate a row-sharded tensor from every rank (variable row counts)."""
    if _SIM is not None:
        return torch.cat([t] * _SIM[1])
    if not is_dist():
        return t
    dev = _comm_device(t)
    x = t.to(dev).contiguous()
    n = torch.tensor([x.shape[0]], device=dev, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world())]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=dev)
    pad[:x.shape[0]] = x
    if x.dtype == torch.bool:
        pad = pad.to(torch.uint8)
    bufs = [torch.empty_like(pad) for _ in range(world())]
    dist.all_gather(bufs, pad)
    out = torch.cat([b[:s] for b, s in zip(bufs, sizes)])
    if x.dtype == torch.bool:
        out = out.to(torch.bool)
    return out.to(t.device)


def all_to_all_bytes(per_dest: Sequence[bytes]) -> List[bytes]:
    """Personalised exchange: rank r sends ``per_dest[k]`` to rank k and returns what every rank sent it
    (two ``all_to_all_single`` calls: the sizes, then the payload with those splits)."""
    if _SIM is not None:
        return [per_dest[_SIM[0]]] * _SIM[1]
    if not is_dist():
        return [per_dest[0]]
    n = world()
    if len(per_dest) != n:
        raise ValueError("one payload per destination rank")
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    send_sizes = torch.tensor([len(b) for b in per_dest], dtype=torch.int64, device=dev)
    recv_sizes = torch.empty_like(send_sizes)
    dist.all_to_all_single(recv_sizes, send_sizes)
    ss, rs = send_sizes.tolist(), recv_sizes.tolist()
    payload = torch.frombuffer(bytearray(b"".join(per_dest)) or bytearray(1), dtype=torch.uint8)[:sum(ss)].to(dev)
    out = torch.empty(sum(rs), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(out, payload, output_split_sizes=rs, input_split_sizes=ss)
    data = out.cpu().numpy().tobytes()
    res, o = [], 0
    for k in rs:
        res.append(data[o:o + k])
        o += k
    return res


def key_owner(key, n: int) -> int:
    """Rank owning a record key: a process-independent hash (crc32 of its string form)."""
    import zlib
    return zlib.crc32(str(key).encode("utf-8")) % n


def shuffle_by_key(records: Sequence, key_fn) -> list:
    """Keyed shuffle (Spark ``reduceByKey`` / ``groupByKey`` exchange): every record goes to
    the rank that owns its key; returns the records this rank owns (from all ranks, rank order)."""
    import pickle
    if not is_dist():
        return list(records)
    n = world()
    buckets: List[list] = [[] for _ in range(n)]
    for r in records:
        buckets[key_owner(key_fn(r), n)].append(r)
    # payloads are this job's own in-memory records exchanged between its ranks
    got = all_to_all_bytes([pickle.dumps(b, protocol=pickle.HIGHEST_PROTOCOL) for b in buckets])
    out: list = []
    for g in got:
        out.extend(pickle.loads(g))
    return out


def lpt_assign(costs: Sequence[float], n_workers: int) -> List[int]:
    """Longest-processing-time-first assignment of tasks to workers; returns worker per task."""
    order = sorted(range(len(costs)), key=lambda i: -costs[i])
    load = [0.0] * n_workers
    owner = [0] * len(costs)
    for i in order:
        w = min(range(n_workers), key=lambda k: load[k])
        owner[i] = w
        load[w] += costs[i]
    return owner
