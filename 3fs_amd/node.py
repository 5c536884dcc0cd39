"""Node scale-out: shard chunks by chain id over the GPUs of a node, hash each
shard locally, all-gather the per-chain digest tables over RCCL (xGMI).

3FS routes every chunk IO by chain (StorageOperator.cc:248-256; GlobalKey
vChainId, src/fbs/storage/Common.h:252-267), and a chunk's checksum depends
only on its own bytes, so the data path needs no inter-GPU exchange at all.
The single collective is the final all-gather of (chunk index, crc) digests
(SURVEY.md §8e): 8 bytes per chunk, latency-bound, far below the xGMI bound.
"""
import numpy as np


def chain_of(chunk_ids, num_chains):
    """Chain id of each chunk for a chain table of `num_chains` chains (round-robin layout)."""
    return np.asarray(chunk_ids, dtype=np.int64) % num_chains


def shard_chunk_ids(n_chunks, rank, world, num_chains=None):
    """Chunk ids owned by `rank`: those whose chain id maps to this GPU (chain % world)."""
    num_chains = num_chains or world
    ids = np.arange(n_chunks, dtype=np.int64)
    return ids[chain_of(ids, num_chains) % world == rank]


def allgather_digests(local_ids, local_crcs, world, group=None):
    """All-gather (chunk id, raw crc) pairs from every rank and return the full
    digest table ordered by chunk id: (ids int64[N], crcs uint32[N]).

    local_ids / local_crcs: torch tensors on the rank's device (CUDA -> RCCL,
    CPU -> gloo).  Ranks may own different chunk counts: rows are padded to the
    largest shard and the padding (id -1) dropped.
    """
    import torch
    import torch.distributed as dist

    dev = local_ids.device
    n_local = torch.tensor([local_ids.numel()], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(counts, n_local, group=group)
    m = int(max(int(c.item()) for c in counts))
    table = torch.full((m, 2), -1, dtype=torch.int64, device=dev)
    table[:local_ids.numel(), 0] = local_ids.to(torch.int64)
    table[:local_ids.numel(), 1] = local_crcs.to(torch.int64) & 0xFFFFFFFF
    parts = [torch.empty_like(table) for _ in range(world)]
    dist.all_gather(parts, table, group=group)
    g = torch.cat(parts).cpu().numpy()
    g = g[g[:, 0] >= 0]
    order = np.argsort(g[:, 0], kind="stable")
    return g[order, 0], g[order, 1].astype(np.uint32)
