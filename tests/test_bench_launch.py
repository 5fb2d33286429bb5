"""bench.py's multi-GPU launch on CPU: `--gpus N` without a launcher starts
N ranks under torch.distributed.run as a child (no GPU is touched; the
SMMD_BENCH_PROBE hook makes each rank report its layout and exit), and a
launcher whose WORLD_SIZE differs from --gpus is refused."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_launch_plan():
    import bench
    assert bench.launch_plan(1, {}) == ('run', 1)
    assert bench.launch_plan(4, {}) == ('spawn', 4)
    assert bench.launch_plan(2, {'WORLD_SIZE': '2'}) == ('run', 2)
    assert bench.launch_plan(1, {'WORLD_SIZE': '1'}) == ('run', 1)
    with pytest.raises(SystemExit):
        bench.launch_plan(8, {'WORLD_SIZE': '2'})
    with pytest.raises(SystemExit):
        bench.launch_plan(1, {'WORLD_SIZE': '4'})
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args,
                          capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)


def test_gpus_2_spawns_two_ranks():
    r = _run(['--gpus', '2', '--steps', '3'], {'SMMD_BENCH_PROBE': '1'})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith('{')]
    assert sorted(x['rank'] for x in lines) == [0, 1]
    assert all(x['world'] == 2 and x['gpus'] == 2 for x in lines)
    assert 'launching 2 ranks' in r.stderr


def test_gpus_mismatch_fails():
    r = _run(['--gpus', '4'], {'SMMD_BENCH_PROBE': '1', 'WORLD_SIZE': '2', 'RANK': '0'})
    assert r.returncode != 0
    assert 'WORLD_SIZE=2' in r.stderr


def test_child_exit_code_propagates():
    r = _run(['--gpus', '2'], {'SMMD_BENCH_PROBE': 'fail'})
    assert r.returncode != 0
    assert 'launching 2 ranks' in r.stderr
