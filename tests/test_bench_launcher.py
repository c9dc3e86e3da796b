"""bench.py --gpus N without torch.distributed.run: the parent starts N rank
processes with the torchrun environment, relays rank 0's JSON line and fails when a rank fails;
under a launcher, --gpus must equal WORLD_SIZE.  CPU only: the ranks here are stub workers."""
import json
import os
import subprocess
import sys
import textwrap

from conftest import ROOT

sys.path.insert(0, ROOT)

STUB = textwrap.dedent("""
    import json, os, sys, time
    import torch.distributed as dist
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    env = {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    fail = int(os.environ.get("STUB_FAIL_RANK", "-1"))
    if r == fail:
        sys.stdout.flush()
        os._exit(3)                # a crashed rank (bench.py's ranks leave through os._exit on error)
    if fail >= 0:
        time.sleep(600)            # a rank stuck while another failed: the launcher must end it
    import torch
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    if r == 0:
        print(json.dumps({"n_gpus": w, "sum": float(t), "env": env}), flush=True)
    dist.destroy_process_group()
""")


def test_launch_ranks_starts_n_ranks_and_relays_rank0(tmp_path):
    import bench
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    out = tmp_path / "out.txt"
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(2, [sys.executable, %r]))" % (ROOT, str(stub)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    with open(out, "w") as f:
        r = subprocess.run([sys.executable, "-c", code], stdout=f, stderr=subprocess.PIPE, text=True, env=env,
                           timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in out.read_text().splitlines() if l.startswith("{")]
    assert len(lines) == 1                       # only rank 0's line on stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["sum"] == 3.0
    assert d["env"]["WORLD_SIZE"] == "2" and d["env"]["RANK"] == "0" and d["env"]["MASTER_ADDR"] == "127.0.0.1"
    assert bench.launch_ranks is not None


def test_launch_ranks_fails_and_ends_the_other_ranks(tmp_path):
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(2, [sys.executable, %r]))" % (ROOT, str(stub)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    env["STUB_FAIL_RANK"] = "1"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])


def test_bench_refuses_gpus_different_from_world_size():
    """Under a launcher (WORLD_SIZE set) --gpus N must equal the world: checked before any GPU call."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr, r.stderr[-2000:]


def test_bench_self_launch_path_is_taken_before_any_gpu_call(tmp_path):
    """`python bench.py --gpus 2` (no WORLD_SIZE) goes through launch_ranks with this same command;
    a stand-in launch_ranks records the command instead of starting GPU ranks."""
    code = textwrap.dedent(f"""
        import json, sys
        sys.path.insert(0, {ROOT!r})
        import bench, torch
        seen = {{}}
        def fake(n, cmd, env=None, poll_s=0.2):
            seen.update(n=n, cmd=cmd, cuda_init=torch.cuda.is_initialized())
            return 0
        bench.launch_ranks = fake
        sys.argv = ["bench.py", "--gpus", "2", "--steps", "3"]
        try:
            bench.main()
        except SystemExit as e:
            seen["exit"] = e.code
        print(json.dumps(seen))
    """)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n"] == 2 and d["exit"] == 0 and d["cuda_init"] is False
    assert d["cmd"][1].endswith("bench.py") and d["cmd"][2:] == ["--gpus", "2", "--steps", "3"]
