"""Device-code guards (CPU) on the gfx950 code objects inside libmpcfatigue.so (read from the clang offload
bundles of the shared object; no GPU needed):

* no device function calls (s_swappc_b64) and no dynamic stack: every kernel is one inlined body;
* no flat access whose immediate offset spans a joint record: the generic solver's kernels read their model
  images in LDS through generic (flat) pointers, and the aperture of a flat access is decided on its base
  register.  A joint loop strength-reduced to `base - 400 k` plus a folded offset put that base below the LDS
  aperture and faulted the line-search kernel (MEMORY_APERTURE_VIOLATION, rounds 3 and 4);
  dyn.hpp joint_at keeps each joint's address a pointer of its own, and this test keeps it so.
"""
import os
import re
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mpc_fatigue_amd", "libmpcfatigue.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _gfx950_objects(path):
    b = open(path, "rb").read()
    out = []
    for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), b):
        st = m.start()
        n = struct.unpack_from("<Q", b, st + 24)[0]
        p = st + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, p)
            p += 24
            triple = b[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size > 0:
                out.append(b[st + off:st + off + size])
    return out


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_no_device_function_calls(tmp_path):
    objs = _gfx950_objects(LIB)
    assert objs, "no gfx950 code object in libmpcfatigue.so"
    calls = 0
    for i, o in enumerate(objs):
        f = tmp_path / f"co{i}.o"
        f.write_bytes(o)
        asm = subprocess.run([OBJDUMP, "-d", str(f)], capture_output=True, text=True, check=True).stdout
        assert "s_endpgm" in asm
        calls += asm.count("s_swappc_b64")
    assert calls == 0, f"{calls} device function calls (s_swappc_b64) in the gfx950 code objects"


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_no_dynamic_stack(tmp_path):
    """No kernel may need a dynamic stack (a call the compiler cannot bound, or recursion): its private segment
    would be sized at run time.  Round 3's aperture-violation kernel had a real call."""
    readelf = os.path.join(os.path.dirname(OBJDUMP), "llvm-readelf")
    checked = 0
    for i, o in enumerate(_gfx950_objects(LIB)):
        f = tmp_path / f"co{i}.o"
        f.write_bytes(o)
        notes = subprocess.run([readelf, "--notes", str(f)], capture_output=True, text=True, check=True).stdout
        kernels = notes.split(".agpr_count:")[1:]
        for k in kernels:
            m = re.search(r"\.name:\s+(\S+)", k)
            if not m:
                continue
            checked += 1
            assert not re.search(r"\.uses_dynamic_stack:\s+true", k), m.group(1)
    assert checked > 0


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_no_flat_offset_across_joint_records(tmp_path):
    """In the generic solver's kernels (mf::k_g*) every flat load / store offset stays inside one joint record
    (sizeof(DevJoint) = 400 bytes, model.hpp): a larger one means a joint address folded into the instruction
    offset, with the base register below the model image (see the module docstring)."""
    worst = {}
    for i, o in enumerate(_gfx950_objects(LIB)):
        f = tmp_path / f"co{i}.o"
        f.write_bytes(o)
        asm = subprocess.run([OBJDUMP, "-d", str(f)], capture_output=True, text=True, check=True).stdout
        cur = None
        for line in asm.split("\n"):
            m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
            if m:
                cur = m.group(1)
                continue
            if cur and re.search(r"\d+k_g", cur):
                m = re.search(r"\bflat_(?:load|store)\w*\s.*?offset:(\d+)", line)
                if m:
                    worst[cur] = max(worst.get(cur, 0), int(m.group(1)))
    assert worst, "no flat access found in the generic kernels"
    bad = {k: v for k, v in worst.items() if v >= 400}
    assert not bad, bad
