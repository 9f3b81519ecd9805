"""The leader backward's split LDS exchange (roi_pool.hip, roi_pool_bwd_lead_kernel):
pair k+1's 16 `ds_read_b64` are issued in one asm statement and waited for in a
later one (`s_waitcnt lgkmcnt(0)` with the same registers as "+v" operands).  The
hardware has no VGPR interlock on LDS returns, so the contract is that nothing
between the issue and the wait reads, copies or overwrites the destination
registers, and that the kernel spills nothing.  This test compiles roi_pool.hip
for gfx950 with the library's flags and checks that contract on the ISA of every
instantiation of the kernel."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "replication_faster_rcnn_amd", "csrc", "roi_pool.hip")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-x", "hip", "--cuda-device-only", "-S"]

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def kernels(asm, name):
    """(symbol, body lines) of every function whose mangled name contains `name`."""
    res = []
    lines = asm.splitlines()
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + name + r"\w*:", l)]
    for i in starts:
        sym = lines[i][:-1].split(":")[0]
        j = i + 1
        while j < len(lines) and "s_endpgm" not in lines[j]:
            j += 1
        res.append((sym, lines[i + 1:j + 1]))
    return res


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm") / "roi_pool.s"
    subprocess.run([HIPCC, *FLAGS, SRC, "-o", str(out)], check=True, capture_output=True, timeout=600)
    return out.read_text()


@pytest.mark.parametrize("name,nread", [("roi_pool_bwd_lead_kernel", 16)])
def test_bwd_kernel_exchange_contract(asm, name, nread):
    """The leader kernel exchanges two RoIs per issue (16 reads)."""
    ks = kernels(asm, name)
    assert ks, f"{name} not found in the ISA"
    checked = 0
    for sym, body in ks:
        code = [l.split(";")[0].strip() for l in body]
        i = 0
        while i < len(code):
            if code[i].startswith("ds_read_b64") and i + nread - 1 < len(code) and \
                    all(code[i + k].startswith("ds_read_b64") for k in range(nread)) and \
                    (i == 0 or not code[i - 1].startswith("ds_read_b64")):
                dst = set()
                for k in range(nread):
                    dst |= regs(code[i + k].split(",")[0])
                j = i + nread
                while j < len(code) and not code[j].startswith("s_waitcnt lgkmcnt(0)"):
                    touched = regs(code[j]) & dst
                    assert not touched, f"{sym}: '{code[j]}' touches exchange registers {sorted(touched)} " \
                                        f"before their s_waitcnt lgkmcnt(0)"
                    j += 1
                assert j < len(code), f"{sym}: exchange issue without a following s_waitcnt lgkmcnt(0)"
                checked += 1
                i = j
            else:
                i += 1
    assert checked > 0, f"no {nread}-read exchange block found"


@pytest.mark.parametrize("name", ["roi_pool_bwd_lead_kernel"])
def test_bwd_kernel_no_scratch(asm, name):
    for sym in {s for s, _ in kernels(asm, name)}:
        m = re.search(r"\.amdhsa_kernel " + re.escape(sym) + r"\n(.*?)\.end_amdhsa_kernel", asm, re.S)
        assert m, sym
        size = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", m.group(1))
        assert size and int(size.group(1)) == 0, f"{sym} uses scratch (spills)"


def test_wave_kernel_no_static_lds(asm):
    """roi_pool_fwd_wave_kernel decodes argmax from absolute LDS byte addresses of its
    dynamic tile, which starts at 0 only while the kernel declares no static
    __shared__: every instantiation's fixed group segment is 0."""
    syms = {s for s, _ in kernels(asm, "roi_pool_fwd_wave_kernel")}
    assert syms, "roi_pool_fwd_wave_kernel not found in the ISA"
    for sym in syms:
        m = re.search(r"\.amdhsa_kernel " + re.escape(sym) + r"\n(.*?)\.end_amdhsa_kernel", asm, re.S)
        assert m, sym
        size = re.search(r"\.amdhsa_group_segment_fixed_size (\d+)", m.group(1))
        assert size and int(size.group(1)) == 0, f"{sym} declares static LDS"
