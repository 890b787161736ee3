"""Group sharding across the GPUs of one node.

FEC groups are independent (`quic_fec_group.cc:338-389` encodes one group from its own
k packets; `:234-297` decodes one group from its own k received packets), so the batch
partitions with no exchange step: rank i owns a contiguous range of groups, runs it on
its own device and stream, and no collective touches the data.  The only collectives are
the timing barrier and the max-over-ranks reduction of the elapsed time.

Two partitions:
  weak   every rank owns `groups_per_rank` groups: rank i -> [i*G, (i+1)*G)  (bench.py)
  strong a fixed global batch split as evenly as possible: [i*T//n, (i+1)*T//n)

Each rank generates its own range's bytes from the global splitmix64 stream
(`quic_amd.synth`) by byte offset, so the union of the shards is byte-identical to the
single-GPU workload of the same total size.
"""


def weak_range(groups_per_rank, rank):
    """(first_group, count) of `rank` under weak scaling."""
    if groups_per_rank < 0 or rank < 0:
        raise ValueError("groups_per_rank and rank must be >= 0")
    return rank * groups_per_rank, groups_per_rank


def strong_range(total_groups, world, rank):
    """(first_group, count) of `rank` when `total_groups` are split over `world` ranks."""
    if world < 1 or not 0 <= rank < world or total_groups < 0:
        raise ValueError("need world >= 1, 0 <= rank < world, total_groups >= 0")
    lo = total_groups * rank // world
    hi = total_groups * (rank + 1) // world
    return lo, hi - lo


def data_byte_offset(first_group, k, block_bytes):
    """Byte offset of group `first_group` in the [G][k][bb] data stream."""
    return first_group * k * block_bytes


def loss_seed(seed, rank):
    """Per-rank seed of the receive-set (loss pattern) generator."""
    return seed + rank


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (identity without an initialised process group).

    Used for the bench's elapsed time: the job is done when the slowest rank is."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64,
                     device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_goodput_gib(groups_per_rank, world, k, payload_bytes, seconds_per_step):
    """Whole-job goodput: all ranks' payload bytes per step / the (max) step time."""
    return groups_per_rank * world * k * payload_bytes / 2**30 / seconds_per_step
