"""bench.py pairs a bench line with profile summaries (profiles/*_kstats.json, *_pmc.json) of the
SAME build and workload only: a summary of another arch or batch must never lend its traffic or
counters to a line (round 5: the BetaVAE-H B=32 line briefly carried the VanillaVAE B=64 traffic,
and IWAE summaries were filtered out as Autoencoder ones because their names contain "ae_")."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _bench():
    import bench
    return bench


def test_profile_workload_from_recorded_arguments():
    b = _bench()
    assert b._profile_workload({"config": ""}) == ("vanilla", 64)
    assert b._profile_workload({"config": "bench.py --steps 20 --warmup 5 "}) == ("vanilla", 64)
    assert b._profile_workload({"config": "--arch betaH --batch 32"}) == ("betaH", 32)
    assert b._profile_workload({"config": "bench.py --steps 20 --arch vq --batch 128"}) == ("vq", 128)


def test_profile_names_select_the_arch_family():
    b = _bench()
    names = lambda arch: {os.path.basename(p) for p in b._profiles("*pmc*.json", arch)}
    van = names("vanilla")
    assert any("iwae_" in n for n in van), "IWAE summaries belong to the VanillaVAE family"
    assert not any(n.startswith(("r4_v6_vq", "r5_v2_vq")) or "_ae_big_" in n for n in van)
    assert all("_vq" in n for n in names("vq"))
    assert all("ae_big" in n for n in names("ae_big"))


def test_matching_profile_requires_the_same_workload():
    b = _bench()
    d = json.load(open(os.path.join(REPO, "profiles", "r5_v2_pmc.json")))
    k = next(iter(d["kernels"]))
    ks = [(None, k)]
    p, _, _ = b._matching_profile("*pmc*.json", "vanilla", ks, d["digest"], 64)
    assert p is not None and os.path.basename(p) == "r5_v2_pmc.json"
    p, _, why = b._matching_profile("*pmc*.json", "vanilla", ks, d["digest"], 48)   # no B=48 summary
    assert p is None and "48" in why


def test_every_profiled_kernel_maps_to_a_gpu_test():
    """tools/kernel_coverage.py over the committed round-6 kernel summaries and coverage records
    (VERDICT r5 #3): every library kernel the benchmarks timed has a passing GPU test that ran it
    at its benched shape."""
    import subprocess
    tool = os.path.join(REPO, "tools", "kernel_coverage.py")
    r = subprocess.run([sys.executable, tool, "--round", "r6"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "0 library kernel(s) without a passing test" in r.stdout
