"""GrowZeroed / ZeroPages (value_type_helpers.h): the host result vectors'
value-initialisation by memmove from the zero page equals resize()
(tests/cpp/grow_zeroed_test.cc; no GPU calls)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "distributed_point_functions_amd", "lib")


def test_grow_zeroed_equals_resize(tmp_path):
    exe = tmp_path / "grow_zeroed_test"
    subprocess.run(["g++", "-O1", "-std=c++20", "-Wall", f"-I{os.path.join(ROOT, 'include')}",
                    os.path.join(ROOT, "tests", "cpp", "grow_zeroed_test.cc"), "-o", str(exe),
                    f"-L{LIB}", "-ldpf", "-ldpf_hip", f"-Wl,-rpath,{LIB}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
