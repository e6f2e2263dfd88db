"""EvaluateUntil's prefix dedup (csrc/host/host_util.h DedupTreeIndices,
distributed_point_function.h:718-742) against a first-seen-order map: the
fused order + count pass over many chunks, orders broken inside a chunk and at
a chunk boundary, random orders, both position types (tests/cpp/dedup_test.cc;
no GPU calls)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "distributed_point_functions_amd", "lib")


def test_dedup_tree_indices(tmp_path):
    exe = tmp_path / "dedup_test"
    subprocess.run(["g++", "-O1", "-std=c++20", "-Wall", "-pthread",
                    f"-I{os.path.join(ROOT, 'include')}",
                    f"-I{os.path.join(ROOT, 'distributed_point_functions_amd', 'csrc', 'host')}",
                    os.path.join(ROOT, "tests", "cpp", "dedup_test.cc"), "-o", str(exe),
                    f"-L{LIB}", "-ldpf", "-ldpf_hip", f"-Wl,-rpath,{LIB}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, DPF_HOST_THREADS="8"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "chunks 8" in r.stdout
    assert "0 failures" in r.stdout
