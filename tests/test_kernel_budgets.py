"""Register / LDS / scratch budgets of the headline gfx950 kernels, read from the code objects embedded in the
in-tree extension (no GPU needed): a compiler update or an edit that spills, or that drops a kernel below the
occupancy its schedule was designed for (2 blocks of 4 waves per CU for the staged 3x3 convolution, one wave per SIMD
for the 4-wave GEMM with its 256 AGPR accumulators, ...), fails here instead of showing up as a slower step."""
import glob
import os
import re
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def _kernels():
    so = glob.glob(os.path.join(ROOT, "k8s_amd", "_C*.so"))
    if not so or not os.path.exists(READELF):
        pytest.skip("extension not built here (python -m k8s_amd._build) or llvm-readelf missing")
    data = open(so[0], "rb").read()
    kern, pos, tmp = {}, 0, os.path.join(ROOT, "build", "budget_co.o")
    os.makedirs(os.path.dirname(tmp), exist_ok=True)
    while True:  # one clang offload bundle per linked object
        i = data.find(b"__CLANG_OFFLOAD_BUNDLE__", pos)
        if i < 0:
            break
        n, off = struct.unpack_from("<Q", data, i + 24)[0], i + 32
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode()
            off += tl
            if "gfx950" not in triple or not sz:
                continue
            with open(tmp, "wb") as f:
                f.write(data[i + o:i + o + sz])
            notes = subprocess.run([READELF, "--notes", tmp], capture_output=True, text=True, check=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk)
                if not name:
                    continue

                def num(key, b=blk):
                    m = re.search(r"\." + key + r":\s+(\d+)", b)
                    return int(m.group(1)) if m else 0

                kern[name.group(1)] = {"agpr": int(re.match(r":\s+(\d+)", blk).group(1)), "vgpr": num("vgpr_count"),
                                       "lds": num("group_segment_fixed_size"),
                                       "scratch": num("private_segment_fixed_size")}
        pos = i + 24
    if os.path.exists(tmp):
        os.remove(tmp)
    assert kern, "no gfx950 kernels found in the extension"
    return kern


def _waves_per_simd(k, threads=256):
    """Occupancy from registers (512 unified VGPRs per SIMD lane, allocated in 8s) and LDS (160 KB per CU)."""
    regs = max(k["vgpr"], 1)
    by_regs = 512 // ((regs + 7) // 8 * 8)
    waves_per_block_per_simd = max(threads // 64 // 4, 1)
    by_lds = (160 * 1024 // k["lds"]) * waves_per_block_per_simd if k["lds"] else 8
    return min(8, by_regs, by_lds)


# kernel-name regex -> (designed waves per SIMD, threads per block)
BUDGETS = [
    (r"c314conv3x3_kernel", 2, 256),
    (r"g414gemm_w4_kernel", 1, 256),
    (r"gemm256r_kernel", 1, 512),
    (r"gsk17gemm_short_kernel", 2, 256),
    (r"3wg3\d*wgrad3x3_kernel|wgrad3x3_kernel", 2, 256),
    (r"stem_conv_fwd_kernel", 2, 256),
    (r"flash_fwd_kernel", 1, 256),
]


def test_no_kernel_uses_scratch():
    bad = {n: k["scratch"] for n, k in _kernels().items() if k["scratch"]}
    assert not bad, bad


@pytest.mark.parametrize("pattern,waves,threads", BUDGETS)
def test_headline_kernel_occupancy(pattern, waves, threads):
    ks = {n: k for n, k in _kernels().items() if re.search(pattern, n)}
    assert ks, pattern
    low = {n[:90]: (k["vgpr"], k["agpr"], k["lds"], _waves_per_simd(k, threads)) for n, k in ks.items()
           if _waves_per_simd(k, threads) < waves}
    assert not low, low


def test_gemm_w4_keeps_its_accumulators_in_agprs():
    """The 4-wave GEMM's 256 x 256 tile lives in 256 AGPRs per lane (the main loop's MFMAs read and write them in
    place): a build that moves them to VGPRs would spill or halve the tile."""
    ks = {n: k for n, k in _kernels().items() if "gemm_w4_kernel" in n}
    assert ks and all(k["agpr"] == 256 for k in ks.values()), {n[:80]: k["agpr"] for n, k in ks.items()}
