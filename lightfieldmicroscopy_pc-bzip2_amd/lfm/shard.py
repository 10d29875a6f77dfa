"""Multi-GPU sharding plan for one stack.

The encode path shards with no data-path collective: the stack's z range is
cut into contiguous slabs whose depths are multiples of the block depth
(default 8, klb_imageHeader.h:88 setDefaultBlockSize), so every bzip2 block
lies wholly inside one slab and a slab's blocks are a contiguous range of the
stack's block ids (ids run x -> y -> z, klb_imageIO.cpp:133-140).  Each GPU
encodes its slab with the predictor chosen on the stack's frame 0 (computed
redundantly on every rank, or broadcast), the slab files are joined with
lfm.merge_slabs, and the result is byte-identical to a one-piece encode.
A slab that starts at an odd frame of a video stack takes its previous raw
frame (z0 - 1) from the caller: no exchange between GPUs.
"""


def plan_slabs(Z, world, block_z=8):
    """[(z0, depth)] for `world` ranks: depths multiples of block_z except the
    last; trailing ranks may get an empty slab when Z is small."""
    if Z <= 0 or world <= 0 or block_z <= 0:
        raise ValueError("Z, world and block_z must be positive")
    nblk = -(-Z // block_z)
    per = -(-nblk // world)
    out = []
    for r in range(world):
        z0 = min(Z, r * per * block_z)
        z1 = min(Z, (r + 1) * per * block_z)
        out.append((z0, z1 - z0))
    return out


def forced_request(chosen, video=False):
    """Header request that forces predictor `chosen` (reference request 8 + k)."""
    if not 0 <= chosen <= 7:
        raise ValueError("predictor must be 0..7")
    return (0x80 if video else 0) | (8 + chosen)


def max_over_ranks(seconds):
    """MAX of a per-rank wall time over the job (the bench's timed region):
    a CUDA tensor under nccl (RCCL), a CPU tensor under gloo; identity when
    torch.distributed is not initialised."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(seconds)
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
