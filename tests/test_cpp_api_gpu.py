"""The C++ template API (include/dpf/*.h) on the GPU: tests/cpp/dpf_api_test.cc
restates the reference's typed two-party reconstruction tests, hierarchical
EvaluateNext, EvaluateAt against EvaluateUntil and DCF Evaluate<T> in C++,
covering the template-only host paths (direct device-to-vector copies of plain
integers, threaded tuple unpacking) that the Python API does not reach."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "distributed_point_functions_amd", "lib", "dpf_api_test")


@pytest.mark.parametrize("overlap_grow", ["1", "0"])
def test_cpp_template_api(overlap_grow):
    # DPF_OVERLAP_GROW: 4-32 MiB results value-initialised on a helper thread
    # during the DMA (default) or chunk by chunk (host_util.h CopyToHostSink);
    # the typed EvaluateUntil / EvaluateAt results of that size (VectorSink and
    # the tuple / IntModN unpacking sink) must be identical either way.
    assert os.path.exists(BIN), "build first: python -m distributed_point_functions_amd.build_native"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, DPF_OVERLAP_GROW=overlap_grow))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
