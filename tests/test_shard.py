"""N>1 path without GPUs: shard planning and the timing reduction over gloo
(world size 2), the same calls and backend bench.py uses on GPUs."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def test_plan_shards_balanced_by_bytes():
    from capnp_packed.shard import plan_shards
    sizes = np.array([512, 32768, 1024, 8192, 8192, 16384, 4, 0, 2048] * 50, dtype=np.uint64)
    swo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    for world in (1, 2, 4, 8):
        b = plan_shards(swo, world)
        assert b[0] == 0 and b[-1] == len(sizes) and (np.diff(b) >= 0).all()
        per = [int(swo[b[r + 1]] - swo[b[r]]) for r in range(world)]
        assert sum(per) == int(swo[-1])
        assert max(per) - min(per) <= 32768 + 1  # within one piece


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from capnp_packed.shard import reduce_max_sum
    mx, sm = reduce_max_sum([1.0 + rank, 10.0 * rank])
    dist.barrier()
    q.put((rank, mx, sm))
    dist.destroy_process_group()


def test_reduce_over_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, mx, sm in got:
        assert mx == [2.0, 10.0] and sm == [3.0, 10.0]


@pytest.mark.parametrize("config,segments", [(2, 48), (3, 12)])
def test_bench_launcher_spawns_ranks(config, segments):
    """bench.py --gpus 2 starts two rank processes itself (no torchrun) and
    drives the shard plan + round trip + max/sum reduction end to end; here
    with the oracle as the kernel (--stub, gloo).  Config 3's ragged messages
    are split by bytes."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "2", "--stub",
                          "--config", str(config), "--segments", str(segments), "--seg-words", "512",
                          "--steps", "2"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["errors"] == 0
    per_msg = 4 if config == 3 else 1
    assert line["pieces_total"] == 2 * segments * per_msg
    b = line["shard_bounds"]
    assert b[0] == 0 and b[-1] == 2 * segments and 0 < b[1] < 2 * segments


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parents[1]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "2", "--stub"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 2
