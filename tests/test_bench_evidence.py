"""bench.py embeds committed counter evidence (profiles/rNN/pmc_traffic.json,
step_flops_pmc.json) only when the file's `smmd_source_hash` stamp equals
the running library's: a file from another build, or without a stamp, is
reported as null with the reason (the BENCH line must not carry
counters of a different tree).  CPU only: no GPU, no library call."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _write(tmp_path, name, d):
    p = tmp_path / name
    p.write_text(json.dumps(d))
    return str(p)


def test_load_stamped_accepts_only_the_running_build(tmp_path):
    import bench
    good = _write(tmp_path, 'a.json', {'smmd_source_hash': 'abc', 'x': 1})
    d, why = bench.load_stamped(good, 'abc')
    assert d == {'smmd_source_hash': 'abc', 'x': 1} and why is None
    d, why = bench.load_stamped(good, 'def')
    assert d is None and 'abc' in why and 'def' in why
    nostamp = _write(tmp_path, 'b.json', {'x': 1})
    d, why = bench.load_stamped(nostamp, 'abc')
    assert d is None and 'no smmd_source_hash' in why
    d, why = bench.load_stamped(str(tmp_path / 'missing.json'), 'abc')
    assert d is None and why.startswith('no ')
    bad = tmp_path / 'c.json'
    bad.write_text('{not json')
    d, why = bench.load_stamped(str(bad), 'abc')
    assert d is None and 'not JSON' in why


def test_pmc_traffic_and_step_counters_refuse_stale(tmp_path, monkeypatch):
    import bench
    pmc = _write(tmp_path, 'pmc.json', {
        'smmd_source_hash': 'old', 'smmd_wino3x3_wgrad': {'traffic_bytes': 123}})
    step = _write(tmp_path, 'step.json', {
        'smmd_source_hash': 'old', 'executed_tflop_per_step': 1.0,
        'executed_tflops_over_busy': 80.0, 'frac_of_fp32_peak_over_busy': 0.5,
        'gpu_busy_ms_per_step': 12.0, 'classes': {}})
    monkeypatch.setattr(bench, 'PMC_TRAFFIC', pmc)
    monkeypatch.setattr(bench, 'STEP_PMC', step)
    t, src, why = bench.pmc_traffic('smmd_wino3x3_wgrad', 'new')
    assert t is None and src is None and 'old' in why
    c = bench.step_counters(12.5, 'new')
    assert c['source'] is None and 'old' in c['null_reason']
    # the same files on the build they were measured with
    t, src, why = bench.pmc_traffic('smmd_wino3x3_wgrad', 'old')
    assert t == 123 and why is None
    t, src, why = bench.pmc_traffic('smmd_adam_flat_sn[D]', 'old')
    assert t is None and 'no smmd_adam_flat_sn[D] group' in why
    c = bench.step_counters(12.5, 'old')
    assert c['smmd_source_hash'] == 'old' and c['executed_tflop_per_step'] == 1.0


def test_committed_profiles_are_stamped():
    """Every counter file bench.py reads is stamped (it may be another build's:
    bench.py then reports null; the stamp itself must be there)."""
    import bench
    for path in (bench.PMC_TRAFFIC, bench.STEP_PMC):
        if os.path.exists(path):
            with open(path) as f:
                assert json.load(f).get('smmd_source_hash'), path
