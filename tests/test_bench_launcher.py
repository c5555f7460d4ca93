"""bench.py --gpus N without torchrun: the parent starts N rank processes itself
(bench.spawn_ranks).  Driven here with a stub worker over gloo on the CPU, so the
launcher's environment contract (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*) and its
exit-code handling are checked without a GPU."""
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = r"""
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
assert r == int(os.environ["RANK"]) == int(os.environ["LOCAL_RANK"])
t = torch.tensor([float(r + 1)])
dist.all_reduce(t)
open(os.path.join(sys.argv[1], f"rank{r}"), "w").write(f"{w} {int(t)}")
dist.barrier()
dist.destroy_process_group()
"""


def test_spawn_ranks_starts_world_size_ranks(tmp_path):
    n = 3
    rc = bench.spawn_ranks(n, [sys.executable, "-c", STUB, str(tmp_path)])
    assert rc == 0
    got = sorted(os.listdir(tmp_path))
    assert got == [f"rank{r}" for r in range(n)]
    for r in range(n):
        w, total = (tmp_path / f"rank{r}").read_text().split()
        assert int(w) == n and int(total) == n * (n + 1) // 2


def test_spawn_ranks_reports_a_failing_rank():
    stub = "import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)"
    assert bench.spawn_ranks(2, [sys.executable, "-c", stub]) == 3


def test_bench_refuses_more_gpus_than_visible():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = ""
    env["CUDA_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "GPU(s) visible" in p.stderr


def test_spawn_ranks_ends_the_job_when_a_later_rank_dies():
    """Rank 1 exits with 3 while rank 0 blocks in a gloo barrier that can never
    complete: the launcher must return 3 promptly (it polls every rank), not wait
    for rank 0's collective timeout."""
    import time
    stub = (
        "import os, sys, datetime, torch.distributed as dist\n"
        "dist.init_process_group('gloo', timeout=datetime.timedelta(seconds=600))\n"
        "if os.environ['RANK'] == '1':\n"
        "    os._exit(3)\n"
        "dist.barrier()\n"
    )
    t0 = time.time()
    rc = bench.spawn_ranks(2, [sys.executable, "-c", stub])
    assert rc == 3
    assert time.time() - t0 < 120


def test_visible_gpus_counts_without_hip(monkeypatch):
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2")
    assert bench.visible_gpus() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus() == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    assert bench.visible_gpus() >= 0      # sysfs count (0 in a container without a GPU)
