"""Multi-GPU path on CPU: utterance sharding + the gloo control plane that
bench.py uses for N > 1 (world_size 2, no GPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from open_universe_amd.sharding import max_over_ranks, shard_utterances


def test_shards_are_a_balanced_partition():
    lengths = [128000, 64000, 96000, 32000, 128000, 16000, 8000, 120000, 64000]
    for w in (1, 2, 3, 4, 8):
        shards = shard_utterances(lengths, w)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(lengths)))
        loads = [sum(lengths[i] for i in s) for s in shards]
        assert max(loads) - min(loads) <= max(lengths)


def test_equal_clips_split_evenly():
    shards = shard_utterances([128000] * 32, 8)
    assert [len(s) for s in shards] == [4] * 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, lengths, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard_utterances(lengths, world)[rank]
    # each rank "processes" its own utterances: here, the sum of their lengths
    work = float(sum(lengths[i] for i in mine))
    dist.barrier()
    total = torch.tensor([work], dtype=torch.float64)
    dist.all_reduce(total)
    mx = max_over_ranks(work)
    q.put((rank, mine, float(total.item()), mx))
    dist.destroy_process_group()


def test_two_rank_gloo_sharding():
    lengths = [128000, 64000, 96000, 32000, 128000, 16000]
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, lengths, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    shards = [r[1] for r in res]
    assert sorted(shards[0] + shards[1]) == list(range(len(lengths)))
    assert not set(shards[0]) & set(shards[1])
    assert res[0][2] == res[1][2] == float(sum(lengths))
    loads = [sum(lengths[i] for i in s) for s in shards]
    assert res[0][3] == res[1][3] == float(max(loads))
