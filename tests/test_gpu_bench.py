"""bench.py's JSON contract on the GPU (one short run per workload shape, as a child
process like the driver's own run): the keys and types the driver and the judge read,
the roofline object, and the result checks."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args):
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *args],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def check_contract(d, steps, warmup):
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step',
              'higher_is_better', 'scaling', 'vs_baseline', 'dtype', 'data', 'config',
              'roofline'):
        assert k in d, k
    assert d['n_gpus'] == 1 and d['steps'] == steps and d['warmup'] == warmup
    assert d['value'] > 0 and d['ms_per_step'] > 0 and d['higher_is_better'] is True
    assert d['scaling'] in ('weak', 'strong') and 'workload' in d['config']
    r = d['roofline']
    for k in ('bound', 'achieved', 'peak', 'unit', 'frac', 'traffic'):
        assert k in r, k
    assert r['bound'] in ('hbm', 'mfma') and r['achieved'] > 0
    assert abs(r['frac'] - r['achieved'] / r['peak']) < 1e-9
    assert d['checks']['replicas_identical'] is True


@pytest.mark.gpu
def test_bench_contract_c1(gpu):
    d = run_bench('--config', 'c1', '--steps', '2', '--warmup', '1', '--no-cpu-baseline')
    check_contract(d, 2, 1)
    assert d['matcher']['kind'] == 'exact' and d['matcher']['full_scans'] == 0


@pytest.mark.gpu
def test_bench_contract_c5_streams(gpu):
    d = run_bench('--config', 'c5', '--jobs', '2', '--batch', '1', '--streams', '2', '--steps', '1',
                  '--warmup', '1', '--no-cpu-baseline')
    check_contract(d, 1, 1)
    assert d['scaling'] == 'weak' and d['config']['streams_per_gpu'] == 2
    assert d['checks']['concurrent_identical'] is True


@pytest.mark.gpu
def test_bench_contract_c5_batch(gpu):
    """c5's default form: the GPU's jobs in one batch (one screen and one fused launch per
    wave serve them all); every job's result equals its own one-job synthesis."""
    d = run_bench('--config', 'c5', '--jobs', '3', '--steps', '1', '--warmup', '1',
                  '--no-cpu-baseline')
    check_contract(d, 1, 1)
    assert d['config']['jobs_per_launch'] == 3 and d['config']['jobs_per_gpu'] == 3
    assert d['checks']['batch_identical'] is True and d['checks']['bp_equals_ap_at_s'] is True


@pytest.mark.gpu
def test_bench_two_ranks_sharing_the_gpu_equal_one_rank(gpu):
    """bench.py --gpus 2 as the driver's multi-GPU run starts it (its own launcher), both
    ranks on the box's one GPU (IA_SHARE_GPU=1) with every c1 level sharded over the
    device-side exchange: one JSON line with n_gpus 2, identical replicas, and the 1-rank
    checksum (the sharded synthesis is exact)."""
    one = run_bench('--config', 'c1', '--steps', '1', '--warmup', '0', '--no-cpu-baseline')
    env = dict(os.environ, IA_SHARE_GPU='1', IA_SHARD_MIN_ROWS='0')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2',
                        '--config', 'c1', '--steps', '1', '--warmup', '0', '--no-cpu-baseline'],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout[-2000:]
    two = json.loads(lines[0])
    assert two['n_gpus'] == 2 and two['config']['parallelism'] == 'db-shard2'
    assert two['config']['exchange'].startswith('peer')
    assert two['checks']['replicas_identical'] is True
    assert two['checks']['checksum'] == one['checks']['checksum']


@pytest.mark.gpu
def test_bench_c4_two_ranks_sharing_the_gpu_equal_one_rank(gpu):
    """c4 itself (A = A' 2048^2, B 1024^2, 5-level cap) as the driver's 2-GPU run starts it,
    both ranks on the box's one GPU: the 4.19 M-row finest DB and the 1 M-row level sharded
    over the device-side exchange, replicas identical, the 1-rank checksum, no fallback."""
    one = run_bench('--config', 'c4', '--steps', '1', '--warmup', '0', '--no-cpu-baseline')
    env = dict(os.environ, IA_SHARE_GPU='1')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2',
                        '--config', 'c4', '--steps', '1', '--warmup', '0', '--no-cpu-baseline',
                        '--strict-exchange'],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout[-2000:]
    two = json.loads(lines[0])
    assert two['n_gpus'] == 2 and two['config']['parallelism'] == 'db-shard2'
    assert two['config']['exchange'].startswith('peer') and 'exchange_fallback' not in two['checks']
    assert two['checks']['replicas_identical'] is True and two['checks']['bp_equals_ap_at_s'] is True
    assert two['checks']['checksum'] == one['checks']['checksum']
    assert two['exchange_fallback'] is None
    for r in two['ranks']:       # each rank explains its exchange and its screen
        assert r['exchanges'] and all(e['kind'] == 'peer' for e in r['exchanges'])
        assert all(e['stress'].startswith('ok') for e in r['exchanges'])
        assert r['checksum'] == one['checks']['checksum'] and r['peer_wait_us_per_pixel'] >= 0
        assert r['kernel'].startswith('k_screen16') and r['screen_avg_us'] > 0
        assert 0 < r['frac'] < 1 and r['pipe_frac'] >= r['frac']


@pytest.mark.gpu
def test_bench_c5_two_ranks_sharing_the_gpu(gpu):
    """c5 (the multi_script batch, multi_script.py:13-32) as the driver's 2-GPU run starts
    it, both ranks on the box's one GPU: n_gpus 2, parallelism jobs2, the pixel accounting
    of the whole job (2 ranks x 3 jobs x 349,184 B' pixels), per-rank fields, and every
    rank's jobs (seeds 1000 + 3 (rank + 2 j)) equal to the same seeds' one-rank run."""
    one = run_bench('--config', 'c5', '--jobs', '6', '--steps', '1', '--warmup', '0',
                    '--no-cpu-baseline')
    env = dict(os.environ, IA_SHARE_GPU='1')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2',
                        '--config', 'c5', '--jobs', '3', '--steps', '1', '--warmup', '0',
                        '--no-cpu-baseline'],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout[-2000:]
    two = json.loads(lines[0])
    assert two['n_gpus'] == 2 and two['config']['parallelism'] == 'jobs2'
    assert two['scaling'] == 'weak'
    assert two['config']['pixels_per_step'] == 2 * 3 * 349184
    assert abs(two['value'] - 2 * 3 * 349184 / (two['ms_per_step'] * 1e-3)) < 1e-6 * two['value']
    ranks = two['ranks']
    assert [r['rank'] for r in ranks] == [0, 1]
    ref = one['checks']['job_sums']
    assert len(ref) == 6
    seen = {}
    for r in ranks:
        assert r['jobs'] == 3 and r['pixels_per_step'] == 3 * 349184
        for seed, v in r['job_sums'].items():
            assert (int(seed) - 1000) // 3 % 2 == r['rank'], (seed, r['rank'])
            seen[seed] = v
    assert seen == ref
