"""World-size-2 gloo run of the sharded decode path on CPU.

Each rank takes its contiguous block of row groups (shard.row_group_block), decodes it (here with
the CPU oracle: there is no GPU in this container; the GPU ranks run the same sharding in bench.py
with RCCL), and the measurement reduction (max time, sum of bytes) runs over gloo.  Rank 0 checks
that the union of the shards is the whole file, in order, bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from conftest import load_package
        from oracle import oracle as O

        shard = load_package().shard
        data = np.fromfile(path, dtype=np.uint8)
        fr = O.FileReader(data)
        rg0, rg1 = shard.row_group_block(len(fr.row_groups), world, rank)
        blobs, nbytes = [], 0
        for rg in range(rg0, rg1):
            for ci in range(len(fr.columns)):
                for r in O.decode_chunk(fr.read_chunk(rg, ci)):
                    assert r.status == 0
                    blobs.append((rg, ci, bytes(r.values)))
                    nbytes += len(r.values)
        t, total = shard.reduce_step(0.5 + rank, nbytes)
        # the bench's exchange: every rank's block, checked to tile the file
        rows = sum(fr.row_group_num_rows(rg) for rg in range(rg0, rg1))
        blocks = shard.gather_blocks(rg0, rg1, rows, nbytes)
        shard.check_cover(blocks, len(fr.row_groups), sum(fr.row_group_num_rows(g) for g in range(len(fr.row_groups))))
        gathered = [None] * world
        dist.all_gather_object(gathered, blobs)
        if rank == 0:
            q.put((t, total, [b for g in gathered for b in g], blocks, shard.global_row_offsets(blocks)))
    finally:
        dist.destroy_process_group()


def test_row_group_block():
    from conftest import load_package

    shard = load_package().shard
    for n in (0, 1, 7, 16, 128):
        for world in (1, 2, 3, 8):
            blocks = [shard.row_group_block(n, world, r) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1
    assert shard.row_offsets([5, 7, 0, 3]) == [0, 5, 12, 12]


def test_two_rank_gloo_shards(tmp_path):
    import fixtures
    from oracle import oracle as O

    W = fixtures.W
    rng = np.random.default_rng(3)
    n = 9000
    data = W.flat([("a", W.Column(W.INT64, rng.integers(0, 1 << 40, n), use_dict=False), W.REQUIRED),
                   ("b", W.Column(W.INT32, rng.integers(0, 50, n).astype(np.int32)), W.REQUIRED)], 1000)
    path = tmp_path / "f.parquet"
    path.write_bytes(data)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(path), q)) for r in range(2)]
    for p in procs:
        p.start()
    t, total, blobs, blocks, offsets = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fr = O.FileReader(np.frombuffer(data, dtype=np.uint8))
    want = []
    for rg in range(len(fr.row_groups)):
        for ci in range(len(fr.columns)):
            for r in O.decode_chunk(fr.read_chunk(rg, ci)):
                want.append((rg, ci, bytes(r.values)))
    assert blobs == want
    assert t == 1.5 and total == sum(len(b[2]) for b in want)
    # the plan the bench uses (shard.row_group_block) for 9 row groups over 2 ranks
    assert [b[:3] for b in blocks] == [(0, 5, 5000), (5, 9, 4000)] and offsets == [0, 5000]
    assert sum(b[3] for b in blocks) == total


def _bench_dry(gpus, *extra):
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dry-run"] + list(extra),
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return json.loads(lines[0])


def test_bench_self_launch_two_ranks():
    """`bench.py --gpus 2` without a launcher starts its two rank processes itself.  The main line is
    C2 at every N (weak scaling: a file per rank, the same per-GPU work as the N=1 line); the
    c3_strong sub-record is C3 (one file of 128 row groups) sharded in contiguous blocks (strong
    scaling).  --dry-run puts the CPU oracle in place of the GPU decode and gloo in place of RCCL, so
    both plans (blocks that tile the file) and the reductions (sum of bytes, max of time) are checked
    here."""
    rows, c3rows, mrows = 20_000, 300_000, 256_000
    d = _bench_dry(2, "--rows", str(rows), "--c3-rows", str(c3rows), "--mixed-rows", str(mrows))
    assert d["dry_run"] and d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["workload"].startswith("C2") and d["config"]["rows_total"] == 2 * rows
    sh = d["shards"]
    assert [s["rank"] for s in sh] == [0, 1] and all(s["rows"] == rows for s in sh)
    assert d["decoded_bytes_total"] == sum(s["decoded_bytes"] for s in sh) and d["max_rank_s"] > 0
    c3 = d["c3_strong"]
    assert c3["scaling"] == "strong" and c3["n_gpus"] == 2 and c3["workload"].startswith("C3")
    assert c3["rows_total"] == c3rows and c3["row_groups"] == 128
    sh = c3["shards"]
    assert sh[0]["row_groups"] == [0, 64] and sh[1]["row_groups"] == [64, 128]
    assert sum(s["rows"] for s in sh) == c3rows
    assert c3["decoded_bytes_total"] == 8 * c3rows == sum(s["decoded_bytes"] for s in sh)
    # mixed_1b at N > 1: north_star's target file (written once, in place, by rank 0) as strong
    # scaling -- the same blocks of its 128 row groups, the whole file covered
    m = d["mixed_1b"]
    assert m["scaling"] == "strong" and m["n_gpus"] == 2 and m["workload"].startswith("mixed")
    assert m["rows_total"] == mrows and m["row_groups"] == 128
    assert [s["row_groups"] for s in m["shards"]] == [[0, 64], [64, 128]]
    assert sum(s["rows"] for s in m["shards"]) == mrows
    assert m["decoded_bytes_total"] == sum(s["decoded_bytes"] for s in m["shards"]) > 42 * mrows


def test_bench_single_gpu_scaling_proxy():
    """At N=1 the c3_strong sub-record carries the single-GPU proxy of the 1->8 curve: the whole C3
    file and rank 0's block of shard.row_group_block(128, N, 0) for N = 2, 4, 8."""
    c3rows = 200_000
    d = _bench_dry(1, "--rows", "10000", "--c3-rows", str(c3rows))
    assert d["n_gpus"] == 1 and d["scaling"] == "weak"
    c3 = d["c3_strong"]
    assert c3["n_gpus"] == 1 and c3["decoded_bytes_total"] == 8 * c3rows
    assert [(p["n_gpus"], p["rank0_row_groups"]) for p in c3["proxy"]] == [(2, [0, 64]), (4, [0, 32]), (8, [0, 16])]
    for p in c3["proxy"]:
        assert abs(p["rank0_decoded_bytes"] * p["n_gpus"] - c3["decoded_bytes_total"]) <= 8 * p["n_gpus"] * 128


def test_bench_strong_main_line():
    """--workload c3 keeps the strong-scaling C3 run as the main line."""
    rows = 300_000
    d = _bench_dry(2, "--workload", "c3", "--rows", str(rows))
    assert d["scaling"] == "strong" and d["config"]["rows_total"] == rows and d["c3_strong"] is None
    assert [s["row_groups"] for s in d["shards"]] == [[0, 64], [64, 128]]


def test_bench_mixed_strong_main_line():
    """--workload mixed: north_star's target file (C2's six columns + C3's DELTA timestamps, 128 row
    groups) as the strong-scaling main line: the blocks of one file tile it across the ranks."""
    rows = 256_000
    d = _bench_dry(2, "--workload", "mixed", "--mixed-rows", str(rows))
    assert d["scaling"] == "strong" and d["config"]["rows_total"] == rows and d["config"]["workload"].startswith("mixed")
    assert [s["row_groups"] for s in d["shards"]] == [[0, 64], [64, 128]]
    assert sum(s["rows"] for s in d["shards"]) == rows
    # every row decodes 4 + 8 + 4 + 1 (def level) + 1 + 16 + 8 bytes, plus 8 per non-null double
    assert d["decoded_bytes_total"] > 42 * rows
