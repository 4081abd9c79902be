"""Multi-GPU sharding of the decode.

Row groups are independent (readRowGroupData, chunk_reader.go:375-404; SeekToRowGroup,
file_reader.go:187-198), so N ranks (one process per GPU) each decode a contiguous block of row
groups with no data-path collective.  Global row offsets come from the footer (host exclusive
scan of RowGroup.NumRows).  The only collectives are the measurement reductions: max of the
per-rank step time, sum of the decoded bytes.
"""


def row_group_block(num_row_groups, world, rank):
    """Contiguous block [rg0, rg1) of row groups for `rank`; sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(num_row_groups, world)
    rg0 = rank * base + min(rank, extra)
    return rg0, rg0 + base + (1 if rank < extra else 0)


def row_offsets(rg_rows):
    """Global first row of every row group (exclusive scan of the footer's NumRows)."""
    out, acc = [], 0
    for n in rg_rows:
        out.append(acc)
        acc += int(n)
    return out


def reduce_step(elapsed_s, decoded_bytes, device=None):
    """Whole-job (max elapsed over ranks, total decoded bytes) over the default process group;
    identity without torch.distributed.  `device` = the tensor device of the backend (a CUDA
    device for nccl/RCCL, None = CPU for gloo)."""
    try:
        import torch
        import torch.distributed as dist
    except Exception:
        return elapsed_s, decoded_bytes
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed_s, decoded_bytes
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    b = torch.tensor([float(decoded_bytes)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return float(t.item()), float(b.item())
