"""Register / scratch audit of the built gfx950 code objects (CPU; reads build/*.o, no GPU).

The kernels that pace their vector-memory queue with hand-counted `s_waitcnt vmcnt(N)` (the LDS-DMA rings of the GEMM
engine, the register-weight convs and the DMA weight gradients) assume a fixed sequence of vector-memory instructions
per tile.  A scratch spill is a vector-memory instruction the count does not know about, so every such kernel that
the product path launches must have no private segment and no VGPR spills; the grouped-epilogue register-weight
convs, which carry their epilogue state (store offsets, masks, output descriptor) across tiles, must not spill SGPRs
either (the grouped masked data gradient spilled 62 / 40 SGPRs and its GB-4 instance produced wrong outputs;
DESIGN §6, round 6).  The production list is the set of counted-vmcnt kernels in the training / C2 / C5 profiles
(profiles/r05c_*kernel_stats.csv).
"""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LLVM = Path("/opt/rocm/lib/llvm/bin")
TOOLS = [shutil.which("objcopy"), LLVM / "clang-offload-bundler", LLVM / "llvm-readelf", shutil.which("c++filt")]

# the counted-vmcnt kernels the product path launches: mangled-name prefixes (c++filt cannot demangle the __bf16
# template arguments) or demangled-name patterns
PRODUCTION = [
    r"^_Z15igemm_pp_kernelI6Conv3AILi128ELb[01]ELi8EE7DenseKCIDF16bLi128ELi8EE6EpiStdIDF16bDF16bDF16bLi4EEE",
    r"^_Z15igemm_pp_kernelI7DenseKCIDF16bLi128ELi8EE7DenseMCIDF16bLi128ELi8EE6EpiStdIDF16bDF16bDF16bLi4EEE",
    r"^_Z15igemm_pp_kernelI7DenseKCIDF16bLi128ELi8EES1_6EpiQKVIDF16bEE",
    r"^_Z15igemm_pp_kernelI7DenseKCIDF16bLi128ELi8EES1_6EpiStdIDF16bDF16bDF16bLi4EEE",
    r"^_Z15igemm_pp_kernelI7DenseKCIDF16bLi128ELi8EES1_6EpiStdIffDF16bLi4EEE",
    r"^_Z15igemm_pp_kernelI7DenseMCIDF16bLi128ELi8EES1_12EpiWgradPartE",
    r"^_Z12igemm_kernelIDF16bLi128ELi128ELi2E",
    r"^_Z12igemm_kernelIDF16bLi256ELi128ELi3E",
    r"^void conv3x3_c64_rw_kernel<(0|2), 64, 2>",
    r"^void conv3x3_c64_rw_kernel<1, (64|96), 0>",
    r"^void conv3x3_c64_rw_kernel<3, 64, 0>",
    r"^void convT4s2_rw_kernel<",
    r"^_Z17conv4s2_rw_kernel",
    r"^_Z24conv4s2_wgrad_dma_kernel",
    r"^void conv3x3_wgrad_dmap_kernel<(false|true), 2>",
]
NO_SGPR_SPILL = [r"^void conv3x3_c64_rw_kernel<(0|2), 64, 2>"]


def _kernels():
    """{(mangled, demangled name): (private_segment_fixed_size, sgpr_spill_count, vgpr_spill_count)} over build/*.o."""
    out = {}
    for obj in sorted((ROOT / "build").glob("*.o")):
        tmp = ROOT / "build" / f".{obj.stem}.fatbin"
        co = ROOT / "build" / f".{obj.stem}.co"
        if subprocess.run([TOOLS[0], "-O", "binary", "--only-section=.hip_fatbin", str(obj), str(tmp)],
                          capture_output=True).returncode or tmp.stat().st_size == 0:
            continue
        subprocess.run([str(TOOLS[1]), "--unbundle", "--type=o", f"--input={tmp}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([str(TOOLS[2]), "--notes", str(co)], check=True, capture_output=True, text=True).stdout
        tmp.unlink()
        co.unlink()
        cur, fields = None, {}
        for line in notes.splitlines():
            m = re.match(r"\s+\.(name|private_segment_fixed_size|sgpr_spill_count|vgpr_spill_count):\s+(\S+)", line)
            if not m:
                continue
            if m.group(1) == "name":
                cur, fields = m.group(2), {}
                continue
            fields[m.group(1)] = int(m.group(2))
            if cur and len(fields) == 3:
                out[cur] = (fields["private_segment_fixed_size"], fields["sgpr_spill_count"], fields["vgpr_spill_count"])
                cur = None
    if out:
        names = list(out)
        dem = subprocess.run([TOOLS[3]], input="\n".join(names), capture_output=True, text=True, check=True).stdout.splitlines()
        out = {(n, d): out[n] for n, d in zip(names, dem)}
    return out


@pytest.fixture(scope="module")
def kernels():
    if not all(t and Path(t).exists() for t in TOOLS):
        pytest.skip("objcopy / clang-offload-bundler / llvm-readelf / c++filt not available")
    if not list((ROOT / "build").glob("*.o")):
        pytest.skip("build/*.o absent: run make (or __graft_entry__.build()) first")
    k = _kernels()
    assert k, "no gfx950 kernels found in build/*.o"
    return k


def test_production_counted_vmcnt_kernels_do_not_spill(kernels):
    seen = set()
    bad = []
    for (mangled, name), (priv, sgpr, vgpr) in kernels.items():
        pats = [p for p in PRODUCTION if re.search(p, mangled) or re.search(p, name)]
        if not pats:
            continue
        seen.update(pats)
        if priv or vgpr or (sgpr and any(re.search(p, name) for p in NO_SGPR_SPILL)):
            bad.append(f"{name[:120]}: private {priv} B, {sgpr} SGPR / {vgpr} VGPR spills")
    assert not bad, "\n".join(bad)
    assert seen == set(PRODUCTION), f"production kernels not found in the build: {set(PRODUCTION) - seen}"


def test_grouped_masked_dgrad_is_not_built(kernels):
    """The grouped masked data-gradient instances (mode 1, GB 2 / 4) and every GB-4 instance are gone."""
    gone = [n for _, n in kernels if re.search(r"^void conv3x3_c64_rw_kernel<(1, \d+, [24]|\d, \d+, 4)>", n)]
    assert not gone, gone
