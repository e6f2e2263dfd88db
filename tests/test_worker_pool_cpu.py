"""The host worker pool (csrc/host/value_type_helpers.cc RunOnPool): nested
parallel loops, exceptions from chunks, concurrent submitters and fork()
(tests/cpp/worker_pool_test.cc; no GPU calls).  ADVICE r5."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "distributed_point_functions_amd", "lib")


def test_worker_pool(tmp_path):
    exe = tmp_path / "worker_pool_test"
    subprocess.run(["g++", "-O1", "-std=c++20", "-Wall", "-pthread",
                    os.path.join(ROOT, "tests", "cpp", "worker_pool_test.cc"), "-o", str(exe),
                    f"-L{LIB}", "-ldpf", "-ldpf_hip", f"-Wl,-rpath,{LIB}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, DPF_HOST_THREADS="8"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
