"""Host-side checks of libsgn's internal arithmetic helpers (CPU only).

sgn::UDiv64 replaces the device's u64 division by the calendar bucket width with a
multiply-high and shifts; it must equal x / d for every u64 x."""
import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parent.parent


def test_udiv64_matches_division(tmp_path):
    exe = tmp_path / "udiv_check"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17",
                    "-I", str(ROOT / "include"), "-I", str(ROOT / "shadow-gen_amd" / "csrc"),
                    str(ROOT / "tests" / "native" / "udiv_check.cpp"), "-o", str(exe)],
                   check=True, capture_output=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert " 0 bad" in out.stdout
