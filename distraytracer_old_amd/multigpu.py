"""Image partition across GPUs and the single exchange step.

Rank r of N renders rows r, r+N, r+2N, ... (interleaved rows balance the
expensive bunny/glass regions); every rank's tile is padded to ceil(H/N) rows
so one `all_gather_into_tensor` (RCCL over xGMI; gloo in CPU tests) brings all
float-RGB tiles to every rank, and `assemble` re-interleaves them.

Pixels, their RNG keys and their per-pixel sample order do not depend on N,
so the assembled image is bit-identical to the 1-GPU image.
"""
from __future__ import annotations


def rows_of(rank: int, world: int, H: int) -> tuple[int, int, int]:
    """(row0, row1, row_step) of a rank's tile."""
    return rank, H, world


def tile_rows(rank: int, world: int, H: int) -> int:
    return len(range(rank, H, world))


def max_tile_rows(world: int, H: int) -> int:
    return (H + world - 1) // world


def assemble(gathered, H: int):
    """gathered: [world, maxrows, W, C] (torch tensor or numpy array) -> [H, W, C]."""
    world, maxrows = gathered.shape[0], gathered.shape[1]
    rest = tuple(gathered.shape[2:])
    full = gathered.swapaxes(0, 1).reshape((maxrows * world,) + rest)  # numpy and torch alike
    return full[:H]


def gather_tiles(tile, dist, group=None):
    """all_gather equal-size padded tiles (tensor [maxrows, W, C]) -> [world, maxrows, W, C]."""
    import torch

    world = dist.get_world_size(group)
    out = torch.empty((world,) + tuple(tile.shape), dtype=tile.dtype, device=tile.device)
    dist.all_gather_into_tensor(out.view(-1), tile.contiguous().view(-1), group=group)
    return out
