"""Multi-GPU sharding of a verification batch, one process per GPU.

Requests are independent, so a batch shards by contiguous request-index range
(SURVEY.md 8(e)); shard boundaries are multiples of 64 so each GPU's accept
bitmask is whole little-endian uint64 words.  The only exchanges are the two
collectives of the path (RCCL over xGMI when the backend is "nccl"):
  C1  all_gather of the bitmask words        -> every rank holds the full mask
  C2  all_reduce(MAX) of uint8 vote ballots  -> set union of distinct voters
Both are a few MB at 16M requests; they are timed separately in bench.py.
"""
import torch
import torch.distributed as dist

from .multi import shard_bounds  # noqa: F401  (64-aligned request-index shards)


def words_per_rank(n, world):
    words = (n + 63) // 64
    return (words + world - 1) // world


def gather_bitmask(local_words, n, group=None):
    """All-gather each rank's bitmask words (int64 tensor of its shard, any
    length <= words_per_rank) into the full mask of ceil(n/64) words."""
    world = dist.get_world_size(group)
    per = words_per_rank(n, world)
    buf = torch.zeros(per, dtype=torch.int64, device=local_words.device)
    buf[: local_words.numel()] = local_words
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    return torch.cat(out)[: (n + 63) // 64]


def union_ballots(ballot, group=None):
    """In-place all_reduce(MAX) of a uint8 ballot tensor (set union)."""
    dist.all_reduce(ballot, op=dist.ReduceOp.MAX, group=group)
    return ballot


class ShardedVerifier:
    """Verify this rank's shard of a device-resident batch and gather the
    full accept mask.  `engine` is this rank's EdVerifyEngine."""

    def __init__(self, engine, group=None):
        self.engine = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0

    def verify(self, d_sig64, d_pk32, d_msgs, d_msg_off, n, stream=None):
        lo, hi = shard_bounds(n, self.world, self.rank)
        m = hi - lo
        words = torch.zeros(max(1, (m + 63) // 64), dtype=torch.int64, device=d_sig64.device)
        if m:
            self.engine.verify_batch_device(d_sig64[lo:hi], d_pk32[lo:hi], d_msgs, d_msg_off[lo:hi + 1], m, words,
                                            stream=stream)
        if self.world == 1:
            return words[: (n + 63) // 64]
        return gather_bitmask(words[: (m + 63) // 64], n, self.group)
