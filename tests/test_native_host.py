"""Host-side checks of libsgn's internal arithmetic helpers (CPU only).

sgn::UDiv64 replaces the device's u64 division by the calendar bucket width with a
multiply-high and shifts; it must equal x / d for every u64 x."""
import pathlib
import subprocess

import pytest

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


def test_message_words_carry_the_tag_in_every_8_bytes(tmp_path):
    """k_rounds_x's round-edge message encoding: a granule is accepted only
    when both of its 8-byte words carry this round's tag, and then decodes to the value."""
    exe = tmp_path / "xh_check"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17",
                    "-I", str(ROOT / "include"), "-I", str(ROOT / "shadow-gen_amd" / "csrc"),
                    str(ROOT / "tests" / "native" / "xh_check.cpp"), "-o", str(exe)],
                   check=True, capture_output=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert " 0 bad" in out.stdout


def _kernel_meta(so):
    """AMDGPU kernel metadata (per kernel: private segment, VGPRs, spills) of every gfx950
    code object bundled into a built library."""
    import re
    import tempfile
    d = pathlib.Path(tempfile.mkdtemp())
    fb = d / "fb.bin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", str(so), str(fb)], check=True)
    data = fb.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)]
    out = {}
    llvm = pathlib.Path("/opt/rocm/lib/llvm/bin")
    for i, o in enumerate(offs):
        b, co = d / f"b{i}.bin", d / f"b{i}.co"
        b.write_bytes(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
        r = subprocess.run([str(llvm / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode:
            continue
        notes = subprocess.run([str(llvm / "llvm-readelf"), "--notes", str(co)], capture_output=True,
                               text=True, check=True).stdout
        # one YAML map per kernel (a list item at two spaces: "  - .agpr_count: ..."); its keys
        # are sorted, so fields such as .group_segment_fixed_size come before .name
        fields = {}
        for line in notes.splitlines():
            if re.match(r"  - \.", line):
                fields = {}
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m:
                out[m.group(1)] = fields
            m = re.match(r"\s+\.(private_segment_fixed_size|group_segment_fixed_size|vgpr_count|vgpr_spill_count):"
                         r"\s+(\d+)", line)
            if m:
                fields[m.group(1)] = int(m.group(2))
    return out


@pytest.mark.skipif(not pathlib.Path("/opt/rocm/lib/llvm/bin/clang-offload-bundler").exists(),
                    reason="ROCm LLVM tools absent")
def test_round_kernels_have_no_scratch():
    # the round kernels must keep every host's state in registers/LDS: a non-inlined helper
    # or a spill puts it in scratch memory and costs ~2x (seen when send_batch was outlined)
    meta = _kernel_meta(ROOT / "shadow-gen_amd" / "libsgn.so")
    # one instantiation per traffic kind; k_rounds also with / without the big-slab path,
    # k_execute per trace mode (traced / lean)
    for k, count in (("k_roundsI", 6), ("k_execute", 6)):
        names = [n for n in meta if k in n]
        assert len(names) == count, names
        for name in names:
            m = meta[name]
            assert m["private_segment_fixed_size"] == 0, (name, m)
            assert m["vgpr_spill_count"] == 0 and m["vgpr_count"] <= 256, (name, m)
    # the persistent multi-shard kernel (one per traffic kind): its exchange state on top of the
    # big-slab path leaves a few spill slots outside the event loop; bounded here
    names = [n for n in meta if "k_rounds_x" in n]
    assert len(names) == 3, names
    for name in names:
        m = meta[name]
        assert m["vgpr_count"] <= 256 and m["private_segment_fixed_size"] <= 256, (name, m)


@pytest.mark.skipif(not pathlib.Path("/opt/rocm/lib/llvm/bin/clang-offload-bundler").exists(),
                    reason="ROCm LLVM tools absent")
def test_round_kernel_lds_budget():
    # config C's persistent grid must stay entirely resident at one group per workgroup: its
    # 1563 host groups need 7 workgroups per CU, i.e. static + dynamic LDS (64-run slabs:
    # 64 x 36 B) within 45 granules of 512 B (7 x 23040 <= 160 KiB). A few dozen bytes more
    # dropped the grid to 1536 and cost 14 % (round 3).
    meta = _kernel_meta(ROOT / "shadow-gen_amd" / "libsgn.so")
    for name, m in meta.items():
        if "k_rounds" in name:
            total = m["group_segment_fixed_size"] + 64 * 32 + 2 * 64 * 2
            assert -(-total // 512) * 512 * 7 <= 160 * 1024, (name, m, total)


@pytest.mark.skipif(not pathlib.Path("/opt/rocm/lib/llvm/bin/clang-offload-bundler").exists(),
                    reason="ROCm LLVM tools absent")
def test_periodic_round_kernel_lds_budget():
    # config D's persistent grid needs 8 workgroups per CU WITH the LDS bucket-minimum table
    # (256 buckets, 128-run slabs): without the table its ~1 M sends a round serialise on a few
    # bucket words (round 4: a 48-record outbox pushed the table out and D ran 3.4x slower)
    meta = _kernel_meta(ROOT / "shadow-gen_amd" / "libsgn.so")
    for name, m in meta.items():
        if "k_roundsILj1E" in name:  # SGN_TRAFFIC_PERIODIC
            runs = 128 * 32 + 2 * 128 * 2
            total = m["group_segment_fixed_size"] + max(runs, 1024) + 257 * 4
            assert -(-total // 512) * 512 * 8 <= 160 * 1024, (name, m, total)


def _periodic_groups(w, P, G):
    """The PERIODIC persistent kernel's group list for workgroup w of P (k_rounds, engine.hip):
    the workgroups sharing w % 8 take one contiguous eighth of the G groups."""
    x = w & 7
    cx = (P - x + 7) >> 3
    before = sum((P - y + 7) >> 3 for y in range(x))
    s0, s1 = G * before // P, G * (before + cx) // P
    return list(range(s0 + (w >> 3), s1, cx))


@pytest.mark.parametrize("P,G", [(1, 1), (2, 5), (7, 7), (9, 100), (625, 625), (2048, 15625),
                                 (1792, 15625), (2040, 15625), (300, 200)])
def test_periodic_xcd_group_mapping_is_a_bijection(P, G):
    # every group exactly once per round, each workgroup's groups inside its XCD class's
    # contiguous range (P > G: the oversized-grid test hook leaves some workgroups idle)
    seen = []
    for w in range(P):
        gs = _periodic_groups(w, P, G)
        assert all(0 <= g < G for g in gs)
        seen += gs
    assert sorted(seen) == list(range(G))
    for x in range(min(8, P)):  # one contiguous range per class
        cls = sorted(g for w in range(x, P, 8) for g in _periodic_groups(w, P, G))
        assert cls == list(range(cls[0], cls[-1] + 1)) if cls else True
