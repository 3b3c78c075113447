"""librae_hip.so is tied to the sources it was built from: build() compiles a hash of the
sources and flags into the library (rae_build_id), rebuilds when that hash differs from the
sources beside it (not on mtimes -- the gitignored .so travels with the tree), and the
Python binding refuses a library built from other sources."""
import os
import shutil
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, os.getcwd())
    import __graft_entry__ as ge
    _lib = ge._lib_mod()
    lib_path = ge.LIB
    print("stale0", ge._stale())
    t0 = os.path.getmtime(lib_path)
    ge.build()                                        # ids match: no rebuild
    print("rebuilt0", os.path.getmtime(lib_path) != t0)
    old = _lib.library_build_id(lib_path)
    hpp = os.path.join(ge.CSRC, "rae_common.hpp")
    with open(hpp, "ab") as fh:                       # flip one byte (append to a comment line)
        fh.write(b"// x\\n")
    print("stale1", ge._stale())
    with open(lib_path, "rb") as fh:
        old_blob = fh.read()
    ge.build()
    new = _lib.library_build_id(lib_path)
    print("ids", old != new, new == _lib.source_build_id())
    with open(lib_path, "wb") as fh:                  # put back a library built from the
        fh.write(old_blob)                            # previous sources
""")

LOAD = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, os.path.join(os.getcwd(), "relation-autoencoder_amd"))
    from rae import _lib
    try:
        _lib.load()
        print("refused False")
    except _lib.RaeError:
        print("refused True")
""")


def test_source_change_triggers_rebuild_and_mismatch_is_refused(tmp_path, built_lib):
    tree = tmp_path / "tree"
    (tree / "relation-autoencoder_amd").mkdir(parents=True)
    shutil.copy(os.path.join(ROOT, "__graft_entry__.py"), tree)
    shutil.copytree(os.path.join(ROOT, "include"), tree / "include")
    for sub in ("csrc", "rae"):
        shutil.copytree(os.path.join(ROOT, "relation-autoencoder_amd", sub),
                        tree / "relation-autoencoder_amd" / sub,
                        ignore=shutil.ignore_patterns("__pycache__"))
    (tree / "check.py").write_text(SCRIPT)
    (tree / "load.py").write_text(LOAD)
    p = subprocess.run([sys.executable, "check.py"], cwd=tree, capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    q = subprocess.run([sys.executable, "load.py"], cwd=tree, capture_output=True, text=True,
                       timeout=120)                   # a fresh process: nothing loaded yet
    assert q.returncode == 0, q.stdout + q.stderr
    out = dict(line.split(" ", 1) for line in (p.stdout + q.stdout).strip().splitlines())
    assert out["stale0"] == "False"
    assert out["rebuilt0"] == "False"
    assert out["stale1"] == "True"
    assert out["ids"] == "True True"
    assert out["refused"] == "True"
