"""tools/dpf_benchmark (the reference's distributed_point_function_benchmark.cc
suite restated against the drop-in C++ API) runs on the GPU: a C++ program
that includes only include/dpf/*.h and links libdpf.so, exercising the
templated EvaluateNext/EvaluateAt/GenerateKeys* entry points the way a
reference user's code does."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "distributed_point_functions_amd", "lib", "dpf_benchmark")


def test_reference_benchmark_suite_small_cases():
    assert os.path.exists(BIN), "build first: python -m distributed_point_functions_amd.build_native"
    flt = ("BM_EvaluateRegularDpf<(uint64_t|XorWrapper<uint128>|Tuple<MyIntModN x5>)>/12|"
           "BM_EvaluateHierarchicalFull<uint32_t>/3|BM_IsrgExampleHierarchy|BM_HeavyHitters/16|"
           "BM_BatchEvaluation<XorWrapper<uint128>>/100/4000|BM_KeyGeneration<true>/128")
    r = subprocess.run([BIN, f"--benchmark_filter={flt}", "--benchmark_min_time=0.01"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = [l.split()[0] for l in r.stdout.splitlines()[1:] if l.startswith("BM_")]
    assert len(rows) == 8, r.stdout
