"""The C restatement (oracle/fmcw_cpu.c), bench.py's CPU baseline and the checker of the
largest GPU parity cases, against the NumPy oracle: map within 1e-5 of the fp64 oracle, and
its CFAR bit-exact with the oracle's CFAR on the same float32 map (1-D, 2-D, override)."""
import numpy as np
import pytest

import fmcw_oracle as O
import cpu_backend as CB
from conftest import rel_err
from fmcw import synth


@pytest.mark.parametrize("ns,nc,nrx,cfar,recipe", [
    (1024, 256, 1, O.Cfar1D(), "two_targets"),
    (256, 128, 2, O.Cfar2D(), "random_target"),
    (128, 64, 1, O.Cfar2D(scale_override=3), "random_target"),
    (512, 32, 1, O.Cfar1D(ref=6, guard=1, rank=9, alpha=3.0), "two_targets"),
])
def test_c_backend_matches_oracle(ns, nc, nrx, cfar, recipe):
    cube = synth.frames(2, ns, nc, nrx, recipe)
    m, d, n = CB.process(cube, cfar, threads=4)
    assert n == len(d)
    for f in range(2):
        ref = O.process(cube[f], None)["mag"]
        assert rel_err(m[f], ref) <= 1e-5
        fn = O.cfar_os1d if isinstance(cfar, O.Cfar1D) else O.cfar_os2d
        det, thr = fn(m[f], cfar)
        np.testing.assert_array_equal(d[d["frame"] == f], O.detections(det, m[f], thr, frame=f))


def test_c_cfar_alone_and_thread_invariance():
    rng = np.random.default_rng(4)
    m = rng.rayleigh(5.0, (3, 96, 64)).astype(np.float32)
    m[1, 40, 10] = 300.0
    m[2, :, ::9] = 80.0
    for cf in (O.Cfar1D(), O.Cfar2D(), O.Cfar2D(scale_override=5)):
        want = np.concatenate([_oracle(m[f], cf, f) for f in range(3)])
        for th in (1, 3, 8):
            np.testing.assert_array_equal(CB.cfar(m, cf, threads=th), want)


def _oracle(m, cf, f):
    det, thr = (O.cfar_os1d if isinstance(cf, O.Cfar1D) else O.cfar_os2d)(m, cf)
    return O.detections(det, m, thr, frame=f)


def test_host_info_fields():
    info = CB.host_info()
    assert info["nproc"] >= 1 and info["affinity"] >= 1 and "cpu_model" in info


def test_c_backend_under_host_sanitizers():
    """oracle/fmcw_cpu.c under AddressSanitizer + UBSan (tools/oracle_asan.sh): whole path and
    CFAR alone at five geometries, 1-D and 2-D, detection capacities shorter than the list."""
    import shutil
    import subprocess
    from conftest import REPO
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    r = subprocess.run(["bash", str(REPO / "tools" / "oracle_asan.sh")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "ok (" in r.stdout
