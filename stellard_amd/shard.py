"""Index sharding of a signature batch over ranks and the accept-bitmap
gather -- the only exchange step of the path.

Partition (same as stl_api.cpp ``shard``): contiguous ranges of whole 64-bit
bitmap words, so every rank writes whole ballot words and its slice of the
byte bitmap starts on a byte boundary.  The gather is one all-gather of
equal-sized int64 word buffers (RCCL over xGMI with backend "nccl"; gloo in
the CPU tests); the per-rank slices are then concatenated and trimmed.
"""
import numpy as np


def shard_range(n, rank, world):
    words = (n + 63) // 64
    per = (words + world - 1) // world
    lo = min(n, rank * per * 64)
    hi = min(n, (rank + 1) * per * 64)
    return lo, hi


def words_per_rank(n, world):
    return ((n + 63) // 64 + world - 1) // world


def gather_bitmap_words(local_words, n, world, dist, group=None):
    """All-gather every rank's bitmap words (padded to words_per_rank) and
    return the full batch's words as one tensor (rank order)."""
    import torch
    per = words_per_rank(n, world)
    buf = torch.zeros(per, dtype=torch.int64, device=local_words.device)
    buf[: local_words.numel()] = local_words
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return torch.cat(parts)[: (n + 63) // 64]


def words_to_bool(words, n):
    arr = words.cpu().numpy() if hasattr(words, "cpu") else np.asarray(words)
    return np.unpackbits(arr.astype("<i8").view(np.uint8), bitorder="little")[:n].astype(bool)


def bool_to_words(bits):
    bits = np.asarray(bits, dtype=bool)
    pad = (-len(bits)) % 64
    b = np.packbits(np.concatenate([bits, np.zeros(pad, bool)]), bitorder="little")
    return b.view("<i8").copy()
