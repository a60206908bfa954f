"""bench.py --gpus N must measure N GPUs: without a launcher it starts
torch.distributed.run as a child process before anything touches a GPU; under a launcher whose
WORLD_SIZE contradicts --gpus it fails loudly.  CPU only: the child is intercepted."""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _args(m, argv):
    saved = sys.argv
    sys.argv = ["bench.py"] + argv
    try:
        return m.parse()
    finally:
        sys.argv = saved


def test_gpus2_without_world_size_starts_torchrun_child(monkeypatch):
    m = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["--gpus", "2", "--steps", "5", "--warmup", "1"]
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    rc = m.self_launch(_args(m, argv), argv)
    assert rc == 7                                   # the child's exit code is the bench's
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv                       # the same flags reach every rank
    assert seen["env"]["MK_BENCH_LAUNCHER"].startswith("bench.py")


def test_launcher_cmd_shape():
    m = _bench()
    a = _args(m, ["--gpus", "8"])
    cmd = m.launcher_cmd(a, ["--gpus", "8"], 29555)
    assert "--nproc-per-node=8" in cmd and "--master-port=29555" in cmd
    assert cmd[-2:] == ["--gpus", "8"]


def test_single_gpu_and_ranks_do_not_relaunch(monkeypatch):
    m = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert m.self_launch(_args(m, []), []) is None                     # N = 1: run in-process
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert m.self_launch(_args(m, ["--gpus", "2"]), ["--gpus", "2"]) is None   # already a rank
    # the end-to-end child inherits WORLD_SIZE from rank 0 and is not a rank itself
    assert m.self_launch(_args(m, ["--e2e-only"]), ["--e2e-only"]) is None


def test_world_size_contradicting_gpus_fails(monkeypatch):
    m = _bench()
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit, match="WORLD_SIZE=4 but --gpus 8"):
        m.self_launch(_args(m, ["--gpus", "8"]), ["--gpus", "8"])
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="--gpus 1"):
        m.self_launch(_args(m, []), [])


def test_process_group_setup_output_stays_off_stdout(capfd):
    """Rank 0's JSON line must be alone on stdout: what C++ prints to fd 1 while the process groups
    are set up ("[Gloo] Rank 0 is connected to ...") goes to stderr."""
    m = _bench()
    with m._stdout_to_stderr():
        os.write(1, b"[Gloo] Rank 0 is connected to 1 peer ranks.\n")
    print('{"metric": 1}')
    out, err = capfd.readouterr()
    assert out == '{"metric": 1}\n' and "[Gloo]" in err


def test_roofline_traffic_profile_matches_the_dominant_kernel():
    """roofline.traffic comes from the committed PMC passes (profiles/pmc_chol_update.json): they must
    be of the kernel the line names (the fused column update) and hold a positive byte count."""
    import json
    m = _bench()
    doc = json.load(open(os.path.join(ROOT, "profiles", "pmc_chol_update.json")))
    assert any(k.startswith("mk::k_chol_update_trsm") for k in doc["instances"])
    assert m._pmc_traffic() == doc["hbm_bytes_per_launch"] > 0
