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


def gather_blocks(rg0, rg1, rows, decoded_bytes, device=None):
    """The one exchange of the sharded decode ("optional final gather"): every
    rank's (first row group, end row group, rows, decoded bytes), all-gathered over the default
    process group (RCCL over xGMI for nccl, gloo on CPU).  A few bytes per rank; identity without
    torch.distributed."""
    mine = (int(rg0), int(rg1), int(rows), int(decoded_bytes))
    try:
        import torch
        import torch.distributed as dist
    except Exception:
        return [mine]
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [mine]
    t = torch.tensor(mine, dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [tuple(int(x) for x in o.tolist()) for o in out]


def check_cover(blocks, num_row_groups, num_rows):
    """The gathered blocks tile [0, num_row_groups) in rank order and their rows sum to the file's."""
    pos = 0
    for rg0, rg1, _, _ in blocks:
        if rg0 != pos or rg1 < rg0:
            raise ValueError(f"row-group blocks do not tile the file: {blocks}")
        pos = rg1
    if pos != num_row_groups or sum(b[2] for b in blocks) != num_rows:
        raise ValueError(f"row-group blocks cover {pos} of {num_row_groups} row groups / "
                         f"{sum(b[2] for b in blocks)} of {num_rows} rows")
    return True


def global_row_offsets(blocks):
    """First global row of every rank's block, from the gathered (rg0, rg1, rows, bytes)."""
    return row_offsets([b[2] for b in blocks])


def decode_sharded(source, devices, columns=None):
    """One process, several GPUs (one host thread + one context per GPU): the row
    groups of `source` are split into contiguous blocks over `devices`, and each block is walked on
    the host and decoded on its device by its own thread (the C-ABI calls release the GIL).
    Returns [(device, rg0, rg1, [reader.ColumnData in (row group, column) order])] in block order.
    A device may appear more than once (several contexts on one GPU)."""
    import threading

    from . import native, reader

    f = native.File(source)
    try:
        cols = list(range(len(f.columns()))) if columns is None else list(columns)
        out = [None] * len(devices)
        errs = []

        def work(k, dev):
            try:
                ctx = native.Context(dev)
                try:
                    rg0, rg1 = row_group_block(f.num_row_groups, len(devices), k)
                    res = reader.decode_chunks(ctx, f, rg0, rg1, cols) if rg1 > rg0 else []
                    out[k] = (dev, rg0, rg1, res)
                finally:
                    ctx.close()
            except Exception as e:  # re-raised in the caller's thread
                errs.append(e)

        threads = [threading.Thread(target=work, args=(k, d)) for k, d in enumerate(devices)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errs:
            raise errs[0]
        return out
    finally:
        f.close()
