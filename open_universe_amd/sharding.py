"""Utterance sharding across GPUs.

Utterances are independent, so N GPUs run N processes that each enhance their
own shard; nothing is exchanged on the data path (no RCCL).  The only
cross-rank traffic is control: a start barrier and a max-reduce of the
elapsed time, over gloo.  A single utterance is never split (the biGRUs and
the global normalisations span the whole clip).
"""
import os


def shard_utterances(lengths, world_size):
    """Longest-processing-time bin packing: returns ``world_size`` lists of
    utterance indices with balanced total length.  Deterministic (ties broken
    by index), so every rank computes the same assignment independently."""
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    order = sorted(range(len(lengths)), key=lambda i: (-lengths[i], i))
    load = [0] * world_size
    shards = [[] for _ in range(world_size)]
    for i in order:
        r = min(range(world_size), key=lambda k: (load[k], k))
        shards[r].append(i)
        load[r] += lengths[i]
    return [sorted(s) for s in shards]


def dist_env():
    """(rank, local_rank, world_size) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def max_over_ranks(value, group=None):
    """Max of a float over all ranks (gloo all_reduce); identity when not
    distributed."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
