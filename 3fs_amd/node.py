"""Node scale-out: shard chunks by chain id over the GPUs of a node, hash each
shard locally, all-gather the per-chain digest tables over RCCL (xGMI).

3FS routes every chunk IO by chain (StorageOperator.cc:248-256; GlobalKey
vChainId, src/fbs/storage/Common.h:252-267), and a chunk's checksum depends
only on its own bytes, so the data path needs no inter-GPU exchange at all.
The single collective is the final all-gather of (chunk id, crc) digests
(SURVEY.md §8e): 8 bytes per chunk, latency-bound, far below the xGMI bound.

Sharding (the one function bench.py, the tests and a node deployment use):
GPU r of G owns the contiguous range of the chain table
[r * C / G, (r + 1) * C / G) (SURVEY.md §8e "contiguous ranges of the chain
table"), so per-GPU work is fixed as G grows (weak scaling) and a rank's
chunks are one contiguous id range when every chunk is its own chain.
"""
import numpy as np


def chain_of(chunk_ids, num_chains):
    """Chain id of each chunk for a chain table of `num_chains` chains (round-robin layout)."""
    return np.asarray(chunk_ids, dtype=np.int64) % num_chains


def chain_range(rank, world, num_chains):
    """[lo, hi): the chain ids GPU `rank` of `world` owns."""
    return rank * num_chains // world, (rank + 1) * num_chains // world


def owner_of_chain(chain_ids, world, num_chains):
    """GPU that owns each chain id (inverse of chain_range)."""
    c = np.asarray(chain_ids, dtype=np.int64)
    return ((c + 1) * world - 1) // num_chains


def shard_chunk_ids(n_chunks, rank, world, num_chains=None):
    """Chunk ids owned by `rank`: those whose chain falls in its chain range.  With
    num_chains = n_chunks (every chunk its own chain, bench.py) the ids are the
    contiguous range [rank * n / world, (rank + 1) * n / world)."""
    num_chains = num_chains or n_chunks
    ids = np.arange(n_chunks, dtype=np.int64)
    lo, hi = chain_range(rank, world, num_chains)
    ch = chain_of(ids, num_chains)
    return ids[(ch >= lo) & (ch < hi)]


def allgather_digests(local_ids, local_crcs, world, group=None, backend=None, shard_size=None):
    """All-gather (chunk id, raw crc) pairs from every rank; returns the node's
    digest table ordered by chunk id as tensors on the ranks' device:
    (ids int64[N], crcs int64[N] holding u32 values).  The table stays where it
    was gathered (HBM under RCCL) and is ordered there (torch.sort).

    Ranks may own different chunk counts: rows are padded to the largest shard
    and the padding (id -1) dropped.  shard_size = every rank's shard size when
    all shards are equal (bench.py): no count exchange and no padding to drop,
    so the gather never waits on the host.  backend
    "gloo" gathers through host memory (the CPU rehearsal of the multi-rank
    logic); the result returns to the device.
    """
    import torch
    import torch.distributed as dist

    dev = local_ids.device
    backend = backend or dist.get_backend(group)
    via_host = backend == "gloo" and dev.type != "cpu"
    cdev = torch.device("cpu") if via_host else dev
    if shard_size is None:
        n_local = torch.tensor([local_ids.numel()], dtype=torch.int64, device=cdev)
        counts = [torch.zeros_like(n_local) for _ in range(world)]
        dist.all_gather(counts, n_local, group=group)
        m = int(max(int(c.item()) for c in counts))
    else:
        m = int(shard_size)
        if local_ids.numel() != m:  # a host-side size: no device sync
            raise ValueError(f"allgather_digests: shard_size={m} but this rank holds {local_ids.numel()} ids; "
                             f"pass shard_size=None for unequal shards")
    table = torch.full((m, 2), -1, dtype=torch.int64, device=dev)
    table[:local_ids.numel(), 0] = local_ids.to(torch.int64)
    table[:local_ids.numel(), 1] = local_crcs.to(torch.int64) & 0xFFFFFFFF
    parts = [torch.empty((m, 2), dtype=torch.int64, device=cdev) for _ in range(world)]
    dist.all_gather(parts, table.to(cdev), group=group)
    g = torch.cat(parts).to(dev)
    if shard_size is None:
        g = g[g[:, 0] >= 0]  # padding rows (a host sync: the result size is data-dependent)
    order = torch.argsort(g[:, 0], stable=True)
    return g[order, 0], g[order, 1]
