"""The C-ABI library builds, loads without a GPU and exports every symbol include/rae.h
declares; the host-only entry points work."""
import ctypes as C
import os
import re

from conftest import ROOT


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "rae.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rae_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_what_binding_expects():
    from rae import _lib
    assert header_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_header_symbol(built_lib):
    for sym in header_symbols():
        assert hasattr(built_lib, sym), sym


def test_struct_layout_matches_header(built_lib):
    from rae import _lib
    cfg = _lib.RaeConfig()
    cfg.decoder, cfg.relations, cfg.embed, cfg.neg_samples = 0, 100, 200, 20
    cfg.batch_size, cfg.world_size = 100, 1
    # record layout (rae_step.hpp): P, dS (m) + V1, V2, dw1, dw2, G1 (r) + coef 2*(2+2s) + loss,
    # 16-B aligned
    rec = built_lib.rae_exchange_record_floats(C.byref(cfg))
    assert rec == ((2 * 100 + 5 * 200 + ((2 * 42 + 3) & ~3) + 1 + 3) & ~3)
    cfg.decoder = 1     # bilinear: + G2, X, Y, A1, A2 (r) + z (m) + aux (4: dOne, c_a1, c_a2)
    assert built_lib.rae_exchange_record_floats(C.byref(cfg)) == \
        ((3 * 100 + 10 * 200 + 4 + ((2 * 42 + 3) & ~3) + 1 + 3) & ~3)
    cfg.decoder = 0
    assert built_lib.rae_exchange_floats(C.byref(cfg)) == rec * 100
    cfg.world_size = 8
    # data parallel, SP: the wire record (no V1 / V2 / G1; + aux (dl, dr) for k_vrec), 692
    # floats instead of 1,288 per example at C3 with dw1 / dw2 in the records ...
    cfg.dp_dense = 1
    wire = (2 * 100 + 2 * 200 + 4 + ((2 * 42 + 3) & ~3) + 1 + 3) & ~3
    assert wire == 692
    assert built_lib.rae_exchange_record_floats(C.byref(cfg)) == wire
    assert built_lib.rae_exchange_floats(C.byref(cfg)) == wire * 800
    # ... or with each rank's dense partial block (2 r m + m floats over its l records)
    cfg.dp_dense = 2
    pc = ((2 * 200 * 100 + 100 + 99) // 100 + 3) & ~3
    part = ((2 * 100 + 4 + ((2 * 42 + 3) & ~3) + 1 + 3) & ~3) + pc
    assert (pc, part) == (404, 696)
    assert built_lib.rae_exchange_record_floats(C.byref(cfg)) == part
    cfg.dp_dense = 0                 # auto: records at l ~ m (the partials would move as much) ...
    assert built_lib.rae_exchange_record_floats(C.byref(cfg)) == wire
    cfg.batch_size = 1024            # ... partials at l >> m: 40 floats of partial block each
    assert built_lib.rae_exchange_record_floats(C.byref(cfg)) == 292 + 40
    cfg.batch_size = 100
    cfg.decoder = 1     # the bilinear decoders exchange their whole record
    assert built_lib.rae_exchange_record_floats(C.byref(cfg)) == \
        ((3 * 100 + 10 * 200 + 4 + ((2 * 42 + 3) & ~3) + 1 + 3) & ~3)
    assert built_lib.rae_version() >= 1


def test_plan_create_rejects_bad_config(built_lib):
    from rae import _lib
    cfg = _lib.RaeConfig()
    cfg.decoder = 7
    bufs = _lib.RaeBuffers()
    h = C.c_void_p()
    rc = built_lib.rae_plan_create(C.byref(cfg), C.byref(bufs), C.byref(h))
    assert rc == -1
    assert b"decoder" in built_lib.rae_last_error()


def test_struct_offsets_match_c_compiler(tmp_path):
    """Every rae_config / rae_buffers field sits at the offset the C compiler gives it."""
    import subprocess
    from rae import _lib
    src = tmp_path / "off.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rae.h"', "int main(void) {"]
    for cname, cls in (("rae_config", _lib.RaeConfig), ("rae_buffers", _lib.RaeBuffers)):
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src.write_text("\n".join(lines))
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = dict(line.rsplit(" ", 1) for line in
               subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
               if line)
    for cname, cls in (("rae_config", _lib.RaeConfig), ("rae_buffers", _lib.RaeBuffers)):
        assert int(got[cname]) == C.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(cls, fname).offset, (cname, fname)


def test_shipped_library_is_not_a_diagnostic_build(built_lib):
    """The in-tree library is the product build: its id is the hash of the sources beside it
    (no -DRAE_DIAG phase-stamp instrumentation, which says 'diag-' in the id), and the kernel
    sources read no environment variables (every kernel form is a rae_config field)."""
    from rae import _lib
    bid = _lib.library_build_id()
    assert bid == _lib.source_build_id()
    assert not bid.startswith("diag")
    for f in _lib.source_files():
        txt = open(f).read()
        assert "getenv" not in txt, f
    # no knockout / instrumentation define in the product flags or the shipped build's command
    flags = " ".join(_lib.BUILD_FLAGS)
    log = os.path.join(ROOT, "relation-autoencoder_amd", "rae", "librae_hip.build.log")
    cmd = open(log).readline() if os.path.exists(log) else ""
    for knob in ("RAE_KO_", "RAE_DIAG", "RAE_STAMPS"):
        assert knob not in flags and knob not in cmd, knob


def test_knockout_knobs_refuse_a_product_build(tmp_path):
    """A timing knockout (-DRAE_KO_*: wrong results) compiles only into a diagnostic build
    (-DRAE_DIAG); the host-side preprocessing pass of a product build stops at the #error."""
    import subprocess
    src = os.path.join(ROOT, "relation-autoencoder_amd", "csrc", "rae.hip")
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-E",
            "--cuda-host-only", src, "-o", str(tmp_path / "pp.i")]
    for knob in ("RAE_KO_C", "RAE_KO_W", "RAE_KO_A"):
        p = subprocess.run(base + [f"-D{knob}=1"], capture_output=True, text=True)
        assert p.returncode != 0 and "timing knockouts" in p.stderr, (knob, p.stderr[-500:])
    p = subprocess.run(base + ["-DRAE_KO_C=1", "-DRAE_DIAG"], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[-500:]


def test_plan_create_rejects_unknown_kernel_form(built_lib):
    from rae import _lib
    cfg = _lib.RaeConfig()
    cfg.decoder, cfg.relations, cfg.embed, cfg.neg_samples = 0, 8, 8, 2
    cfg.batch_size, cfg.world_size, cfg.n_examples = 4, 1, 8
    cfg.sp_forward = 9
    bufs = _lib.RaeBuffers()
    h = C.c_void_p()
    assert built_lib.rae_plan_create(C.byref(cfg), C.byref(bufs), C.byref(h)) == -1
    assert b"kernel form" in built_lib.rae_last_error()
