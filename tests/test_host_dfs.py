"""CPU: the host DFS renderer (saln::render_blocks, the text of render
batches and of the CLI) against the oracle's literal DFS text, compiled
against the in-tree libsaln.so and the oracle library (tests/host/dfs_check.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_render_blocks_equals_literal_dfs(tmp_path):
    from oracle import refcpu
    refcpu.build()
    lib = os.path.join(ROOT, "sequencealigning_amd")
    orc = os.path.join(ROOT, "oracle", "_build")
    exe = str(tmp_path / "dfs_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I" + os.path.join(lib, "csrc"), "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "host", "dfs_check.cpp"), "-L" + lib, "-lsaln",
                    "-L" + orc, "-lrefcpu", "-L/opt/rocm/lib", "-lamdhip64",
                    f"-Wl,-rpath,{orc}:/opt/rocm/lib:{lib}", "-o", exe], check=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
