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


# Rows per step of the device-resident verify time (one main-kernel wave per
# SIMD: 256 CUs x 4 SIMDs x 64 lanes on MI355X); stl_api.cpp g_shard_quantum
QUANTUM = 65536


def shard_range_bytes(lens, rank, world, quantum=QUANTUM):
    """Byte-balanced shard (same as stl_api.cpp shard_bytes_bounds /
    stl_shard_range_bytes): boundary r is the 64-aligned row at or after the
    first row where the byte prefix sum reaches r/world of the total, moved to
    the nearest multiple of ``quantum`` rows when that moves its byte prefix by
    at most 2.5 % of one rank's share.  Variable-length rows (config 5: 100 B -
    4 KB preimages) cost in proportion to their SHA-512 blocks, so ranks get
    equal bytes, not equal counts -- but the verify time rises in steps of
    ``quantum`` rows, so a shard just past a step is pulled back to it."""
    lens = np.asarray(lens, dtype=np.uint64)
    n = lens.shape[0]
    total = int(lens.sum())
    csum = np.concatenate([np.zeros(1, np.uint64), np.cumsum(lens, dtype=np.uint64)])  # csum[i] = sum(lens[:i])

    def bound(r):
        if r <= 0:
            return 0
        if r >= world:
            return n
        target = total * r // world
        # smallest i with prefix(i) = sum(lens[:i]) >= target
        i = 0 if target == 0 else int(np.searchsorted(csum[1:], target, side="left")) + 1
        b = min(n, (i + 63) // 64 * 64)
        q = quantum
        if q >= 64 and q % 64 == 0 and n > q:
            down = b // q * q
            up = down + q
            c = down if (b - down <= up - b or up > n) else up
            if 0 < c < n and abs(int(csum[c]) - target) * world * 40 <= total:
                b = c
        return b

    b = [bound(0)]
    for r in range(1, world + 1):
        b.append(max(b[-1], bound(r)))
    return b[rank], b[rank + 1]


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


def gather_bitmap_words_v(local_words, bounds, dist, group=None):
    """Gather for unequal (byte-balanced) shards: rank r holds the words of
    rows [bounds[r], bounds[r+1]) (every bound a multiple of 64 or the end).
    Pads every slice to the largest, all-gathers, and places slice r at word
    bounds[r] // 64.  The same placement libstl's grouped send/recv gather
    uses (stl_api.cpp gather_to_host)."""
    import torch
    world = len(bounds) - 1
    n = bounds[-1]
    per = max(1, max((bounds[r + 1] - bounds[r] + 63) // 64 for r in range(world)))
    buf = torch.zeros(per, dtype=torch.int64, device=local_words.device)
    buf[: local_words.numel()] = local_words
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = torch.zeros((n + 63) // 64, dtype=torch.int64, device=local_words.device)
    for r in range(world):
        w = (bounds[r + 1] - bounds[r] + 63) // 64
        out[bounds[r] // 64: bounds[r] // 64 + w] = parts[r][:w]
    return out


def words_to_bool(words, n):
    arr = words.cpu().numpy() if hasattr(words, "cpu") else np.asarray(words)
    return np.unpackbits(arr.astype("<i8").view(np.uint8), bitorder="little")[:n].astype(bool)


def bool_to_words(bits):
    bits = np.asarray(bits, dtype=bool)
    pad = (-len(bits)) % 64
    b = np.packbits(np.concatenate([bits, np.zeros(pad, bool)]), bitorder="little")
    return b.view("<i8").copy()
