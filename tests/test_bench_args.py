"""CPU: bench.py's launch logic -- `--gpus N` without an external launcher starts the N ranks itself
(torch.distributed.run, 127.0.0.1) before anything touches the GPU; a launcher's WORLD_SIZE that
disagrees with --gpus is refused."""
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launch_command_shape():
    cmd = bench.launch_command(4, ["--gpus", "4", "--steps", "5"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[cmd.index("--nnodes=1") + 1:cmd.index("--nnodes=1") + 1] == []
    assert os.path.basename(cmd[-5]) == "bench.py" and cmd[-4:] == ["--gpus", "4", "--steps", "5"]


def test_world_size_mismatch_refused():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE=3 but --gpus 2" in r.stderr


def test_launch_ranks_keeps_only_the_json_line_on_stdout(monkeypatch, capsys):
    """The self-launch forwards the ranks' stdout: the JSON line stays on stdout, a backend's chatter
    ("[Gloo] Rank 0 is connected ...") goes to stderr; the launcher's exit status is returned."""
    child = "print('[Gloo] Rank 0 is connected to 1 peer ranks'); print('{\"value\": 1}'); raise SystemExit(3)"
    monkeypatch.setattr(bench, "launch_command", lambda n, argv, port: [sys.executable, "-c", child])
    rc = bench.launch_ranks(2, [])
    out, err = capsys.readouterr()
    assert rc == 3 and out.strip() == '{"value": 1}' and "[Gloo]" in err
