"""ISA checks on the gfx950 code object inside the built librae_hip.so (CPU only: the offload
bundle is extracted and disassembled with the ROCm LLVM tools, no GPU needed).

LDS-DMA (global_load_lds_*) takes its LDS destination from M0.  The C3 forward issues its A-row
DMAs from inline asm (rae_sp.hpp dma_row16) so the compiler's wait-count pass does not see them;
M0 is a reserved register, so the asm saves and restores it instead of clobbering it.  These
tests pin, in the machine code that ships, that every LDS-DMA of the C3 forward has its own M0
write earlier in the same basic block (no branch in between), separated from the DMA by a wait
state, and that the asm hands M0 back (the value it saved) right after the DMA."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(ROOT, "relation-autoencoder_amd", "rae", "librae_hip.so")
BUILD_LOG = os.path.join(ROOT, "relation-autoencoder_amd", "rae", "librae_hip.build.log")
C3_FWD = "_Z9k_forwardILb1EN3rae7FixDimsILi100ELi200ELi20EEEEvNS0_8StepArgsE"


def _tool(name):
    p = os.path.join(LLVM, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not available")
    return p


@pytest.fixture(scope="module")
def disasm(built_lib, tmp_path_factory):
    d = tmp_path_factory.mktemp("isa")
    fat, co = d / "fat.bin", d / "gfx950.co"
    subprocess.run([_tool("llvm-objcopy"), "-O", "binary", "--only-section=.hip_fatbin", LIB,
                    str(fat)], check=True)
    subprocess.run([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    out = subprocess.run([_tool("llvm-objdump"), "-d", str(co)], check=True, capture_output=True,
                         text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is not None and line.startswith("\t"):
            cur.append(line.split("//")[0].strip())
    return funcs


def _writes_m0(ins):
    parts = ins.replace(",", " ").split()
    return len(parts) > 1 and parts[0].startswith("s_") and parts[1] == "m0"


def _ends_block(ins):
    op = ins.split()[0] if ins else ""
    return op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm"))


def _lds_dma_sites(code):
    return [i for i, ins in enumerate(code) if ins.startswith("global_load_lds")]


def test_c3_forward_lds_dma_has_its_own_m0(disasm):
    code = disasm.get(C3_FWD)
    assert code, "the C3 forward kernel is not in the code object"
    sites = _lds_dma_sites(code)
    # one DMA per A row of the example: 1 + 2s = 41 rows over waves 4..7 (unrolled)
    assert len(sites) >= 11, len(sites)
    for i in sites:
        j = i - 1
        while j >= 0 and not _writes_m0(code[j]):
            assert not _ends_block(code[j]), f"branch between M0 write and LDS-DMA at {i}"
            j -= 1
        assert j >= 0, f"no M0 write before the LDS-DMA at {i}"
        assert code[j].startswith("s_mov_b32 m0,"), code[j]
        # the M0 -> LDS-DMA hazard needs one wait state (the asm's s_nop; the compiler's own
        # sites in the general fallback path put address arithmetic there)
        assert i - j >= 2, "no wait state after the M0 write"


def test_c3_forward_asm_restores_m0(disasm):
    """dma_row16: s_mov_b32 sX, m0 ; s_mov_b32 m0, sY ; s_nop ; global_load_lds ; s_mov_b32 m0, sX"""
    code = disasm[C3_FWD]
    asm_sites = [i for i in _lds_dma_sites(code) if code[i - 1].startswith("s_nop")]
    assert len(asm_sites) >= 11, len(asm_sites)     # (NR + 3) / 4 per wave, unrolled
    for i in asm_sites:
        save = code[i - 3].replace(",", " ").split()
        restore = code[i + 1].replace(",", " ").split()
        assert save[:1] == ["s_mov_b32"] and save[2] == "m0", code[i - 3]
        assert restore[:2] == ["s_mov_b32", "m0"] and restore[2] == save[1], (code[i - 3], code[i + 1])


def test_every_lds_dma_follows_an_m0_write(disasm):
    """Every LDS-DMA in the library (compiler-emitted builtins included) has an M0 write earlier
    in its function."""
    n = 0
    for name, code in disasm.items():
        for i in _lds_dma_sites(code):
            assert any(_writes_m0(c) for c in code[:i]), name
            n += 1
    assert n > 0


def test_build_is_warning_free(built_lib):
    """__graft_entry__.build() keeps the compiler's output next to the library."""
    if not os.path.exists(BUILD_LOG):
        pytest.skip("library built without a log (prebuilt)")
    log = open(BUILD_LOG).read()
    assert "warning:" not in log, log[:2000]


P2P_PUSHES = ("_Z10k_p2p_rowsN3rae8StepArgsE", "_Z10k_p2p_recsN3rae8StepArgsE",
              "_Z9k_p2p_preN3rae8StepArgsEii")


def _pending_store_at_end(lines):
    """Forward dataflow over the kernel's control-flow graph: is there a path from a
    store (global_ / buffer_) to s_endpgm with no `s_waitcnt vmcnt(0)` in between?"""
    addrs = [a for a, _ in lines]
    index = {a: k for k, a in enumerate(addrs)}
    succ = []
    for k, (a, ins) in enumerate(lines):
        op = ins.split()[0]
        nxt = [k + 1] if k + 1 < len(lines) else []
        if op.startswith(("s_branch", "s_cbranch")):
            imm = int(ins.split()[1])
            imm = imm - 65536 if imm >= 32768 else imm
            tgt = index.get(a + 4 + 4 * imm)
            assert tgt is not None, ins
            nxt = [tgt] if op == "s_branch" else nxt + [tgt]
        elif op == "s_endpgm":
            nxt = []
        succ.append(nxt)
    pending = [False] * len(lines)
    seen = [False] * len(lines)
    work = [0]
    seen[0] = True
    while work:
        k = work.pop()
        ins = lines[k][1]
        out = pending[k]
        if ins.startswith(("global_store", "buffer_store")):
            out = True
        elif ins.startswith("s_waitcnt") and "vmcnt(0)" in ins:
            out = False
        if ins.startswith("s_endpgm") and pending[k]:
            return True
        for j in succ[k]:
            if not seen[j] or (out and not pending[j]):
                seen[j] = True
                pending[j] = pending[j] or out
                work.append(j)
    return False


@pytest.fixture(scope="module")
def disasm_addr(built_lib, tmp_path_factory):
    d = tmp_path_factory.mktemp("isa_addr")
    fat, co = d / "fat.bin", d / "gfx950.co"
    subprocess.run([_tool("llvm-objcopy"), "-O", "binary", "--only-section=.hip_fatbin", LIB,
                    str(fat)], check=True)
    subprocess.run([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    out = subprocess.run([_tool("llvm-objdump"), "-d", str(co)], check=True, capture_output=True,
                         text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        m = re.match(r"^\t(.+?)\s*//\s*([0-9A-Fa-f]+):", line)
        if cur is not None and m:
            cur.append((int(m.group(2), 16), m.group(1).strip()))
    return funcs


def test_p2p_pushes_store_write_through_at_system_scope(disasm_addr):
    """rae_p2p.hpp "Visibility across GPUs", producer side: every store of the push kernels
    into a peer's memory is a system-scope write-through (sc0 sc1), and no path of the kernel
    reaches s_endpgm with a store not yet waited for (vmcnt(0)) -- no pushed byte is left dirty
    in one of this GPU's L2s, or in flight, when the signal kernel that follows runs."""
    for name in P2P_PUSHES:
        lines = disasm_addr.get(name)
        assert lines, f"{name} is not in the code object"
        stores = [c for _, c in lines if c.startswith(("global_store", "buffer_store"))]
        assert stores, name
        for c in stores:
            assert re.search(r"\bsc0\b", c) and re.search(r"\bsc1\b", c), c
        assert not _pending_store_at_end(lines), name


def test_no_inline_asm_vector_stores():
    """Every vector-memory store of the kernels is one the compiler emits (a plain store or a
    buffer-store builtin), never an inline-asm store: the compiler's hazard and wait-count
    passes do not see inline asm, and an inline-asm store they cannot see let them reuse or wait
    wrongly around it (measured: asm `sc1` row stores in the update gave non-finite costs, the
    same stores as builtins did not -- profiles/r06_ab.txt).  The one inline-asm memory operation
    kept, the forward's LDS-DMA load, is covered by the M0 tests above."""
    csrc = os.path.join(ROOT, "relation-autoencoder_amd", "csrc")
    bad = []
    for fn in sorted(os.listdir(csrc)):
        if not fn.endswith((".hip", ".hpp")):
            continue
        text = open(os.path.join(csrc, fn)).read()
        for m in re.finditer(r"asm\s+volatile\s*\((.*?)\)\s*;", text, re.S):
            if re.search(r"(global|buffer|flat)_store", m.group(1)):
                bad.append(f"{fn}: {m.group(0)[:80]}")
    assert not bad, bad
