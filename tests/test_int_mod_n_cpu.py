"""The drop-in IntModN / Tuple headers against the reference's own unit tests
(dpf/int_mod_n_test.cc:32-254 restated in tests/cpp/int_mod_n_test.cc): the
static sampling API (IntModNBase::GetSecurityLevel / CheckParameters /
GetNumBytesRequired / ConvertBytesTo, IntModN::GetNumBytesRequired /
UnsafeSampleFromBytes / SampleFromBytes) with the reference's Status
messages, the 2^32-5 sampling chain, and constexpr operators."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "distributed_point_functions_amd", "lib")


def test_int_mod_n_reference_unit_tests(tmp_path):
    exe = tmp_path / "int_mod_n_test"
    subprocess.run(["g++", "-O1", "-std=c++20", "-Wall", f"-I{os.path.join(ROOT, 'include')}",
                    os.path.join(ROOT, "tests", "cpp", "int_mod_n_test.cc"), "-o", str(exe),
                    f"-L{LIB}", "-ldpf", "-ldpf_hip", f"-Wl,-rpath,{LIB}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
