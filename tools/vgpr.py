"""Register / scratch / LDS metadata of the round kernels for an engine.hip build variant.
usage: python tools/vgpr.py [-DNAME=VAL ...]   (compiles engine.hip to /tmp, CPU only)"""
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests"))
from test_native_host import _kernel_meta  # noqa: E402

csrc = ROOT / "shadow-gen_amd" / "csrc"
obj = pathlib.Path("/tmp/vgpr_engine.o")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                "-Wno-unused-result", "-Wno-unused-value", f"-I{ROOT / 'include'}", f"-I{csrc}", *sys.argv[1:],
                "-c", str(csrc / "engine.hip"), "-o", str(obj)], check=True)
for k, v in sorted(_kernel_meta(obj).items()):
    if "k_rounds" in k or "k_execute" in k:
        print(f"{k[:44]:44s} vgpr {v['vgpr_count']:3d} spill {v['vgpr_spill_count']} scratch "
              f"{v['private_segment_fixed_size']} lds {v['group_segment_fixed_size']}")
