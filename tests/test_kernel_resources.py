"""CPU: the gfx950 code objects inside libs2lincheck.so, read back from their
metadata notes (no GPU). The search kernels must keep their working state in
registers: a private (scratch) segment on a hot kernel means the compiler
spilled an array to memory, as the level search's move selection did until
round 3 (5.7 GB of scratch writes per C5 search)."""
import os
import re
import subprocess
import tempfile

import pytest

import s2_verification_amd as s2

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


CTL = re.compile(r"\bs_(cbranch_\w+|branch|swappc_b64|setpc_b64)\b")


def frame_scratch_violations(body):
    """Scratch instructions of a called function (its disassembly lines) that
    are not part of its call frame. Allowed: in the prologue (before the first
    branch or call) the callee-saved register saves (stores at fixed s33
    offsets) and the reads of a by-value argument the caller wrote (loads);
    in the epilogue (the straight-line block ending at s_setpc_b64) the
    restores, each of a register the prologue saved, from the same offset.
    Returns the offending lines (empty: the frame is exactly that)."""
    ctl = [i for i, l in enumerate(body) if CTL.search(l)]
    first = ctl[0] if ctl else len(body)

    def in_epilogue(i):  # the straight-line block from i to an s_setpc_b64 (a return)
        nxt = [c for c in ctl if c > i]
        return bool(nxt) and "s_setpc_b64" in body[nxt[0]]

    saved, bad = set(), []
    for i, l in enumerate(body):
        if "scratch_" not in l:
            continue
        m = re.search(r"scratch_(store|load)_dword\s+(?:off, )?(v\d+)(?:, off)?, (s33)(?: offset:(\d+))?", l)
        if m and m.group(1) == "store" and i < first:
            saved.add((m.group(2), m.group(4) or "0"))
        elif "scratch_load" in l and i < first and not m:
            pass  # the by-value argument, read once at entry
        elif m and m.group(1) == "load" and in_epilogue(i) and (m.group(2), m.group(4) or "0") in saved:
            pass
        else:
            bad.append(l.strip())
    return bad


def call_arg_scratch_violations(body):
    """Scratch instructions of a kernel that are not the writes of a by-value
    argument right before a call: every one must be a store inside the
    straight-line block that ends with an s_swappc_b64 (no load at all)."""
    ctl = [i for i, l in enumerate(body) if CTL.search(l)]
    bad = []
    for i, l in enumerate(body):
        if "scratch_" not in l:
            continue
        nxt = [c for c in ctl if c > i]
        if not ("scratch_store" in l and nxt and "s_swappc_b64" in body[nxt[0]]):
            bad.append(l.strip())
    return bad


def kernel_metadata(disasm=False):
    """{kernel name: {'scratch': bytes per lane, 'vgpr': count}} over every
    offload bundle in the library's .hip_fatbin section; with disasm, also
    'scratch_ops' (scratch instructions in the kernel's own code),
    'calls' (s_swappc_b64 in it) and, for every called function (a symbol
    that is not a kernel), 'frame_violations' (frame_scratch_violations)."""
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not all(os.path.exists(t) for t in tools):
        pytest.skip("ROCm LLVM tools not found")
    objcopy, bundler, readelf = tools
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fatbin")
        subprocess.run([objcopy, "--dump-section=.hip_fatbin=" + fat, s2.LIB_PATH, os.path.join(d, "x.so")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        assert starts, "no offload bundle in .hip_fatbin"
        for k, a in enumerate(starts):
            part = os.path.join(d, f"b{k}")
            with open(part, "wb") as f:
                f.write(data[a:starts[k + 1] if k + 1 < len(starts) else len(data)])
            co = os.path.join(d, f"b{k}.co")
            subprocess.run([bundler, "--unbundle", "--type=o", "--input=" + part, "--targets=" + TARGET,
                            "--output=" + co], check=True, capture_output=True)
            notes = subprocess.run([readelf, "--notes", co], check=True, capture_output=True, text=True).stdout
            name = None
            for line in notes.splitlines():
                m = re.match(r"\s*\.name:\s+(\S+)", line)
                if m:
                    name = m.group(1)
                    out.setdefault(name, {})
                m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
                if m and name:
                    out[name]["scratch"] = int(m.group(1))
                m = re.match(r"\s*\.vgpr_count:\s+(\d+)", line)
                if m and name:
                    out[name]["vgpr"] = int(m.group(1))
            if disasm:
                objdump = os.path.join(LLVM, "llvm-objdump")
                text = subprocess.run([objdump, "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                                      text=True).stdout
                cur, body = None, []

                def flush():
                    if cur in out:
                        out[cur]["scratch_ops"] = sum(1 for l in body if "scratch_" in l)
                        out[cur]["calls"] = sum(1 for l in body if "s_swappc" in l)
                        out[cur]["call_arg_violations"] = call_arg_scratch_violations(body)
                    elif cur:
                        out.setdefault("functions", {})[cur] = {
                            "scratch_ops": sum(1 for l in body if "scratch_" in l),
                            "frame_violations": frame_scratch_violations(body)}
                for line in text.splitlines():
                    m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
                    if m:
                        flush()
                        cur, body = m.group(1), []
                    elif cur:
                        body.append(line)
                flush()
    return out


def test_search_kernels_use_no_scratch():
    md = kernel_metadata(disasm=True)
    hot = {n: v for n, v in md.items() if n != "functions" and
           re.search(r"(pack_kernel|search_kernel|lv_round|lv_insert|lv_persist|literal_kernel)", n)}
    assert len(hot) >= 30, sorted(hot)
    for n, v in hot.items():
        # lv_persist runs its solo rounds in noinline functions (lv_solo_wave
        # and its rare paths, solo_dev.h: their own register allocation). Its
        # only scratch instructions are the writes of lv_solo_wave's by-value
        # argument right before the call; the callees' frames are checked
        # exactly below. Round 4's two-per-CU bound had left lv_persist<5>
        # ~300 scratch accesses in its grid rounds. lv_insert
        # declares a 20-byte frame its body never touches (the round close's
        # counters, addressed flat). Every other hot kernel: no scratch at all.
        if "lv_persist" in n:
            assert v.get("call_arg_violations") == [], (n, v["call_arg_violations"][:8])
            # (solo rounds are compiled for NQ <= 5: the others make no call)
            assert v.get("vgpr", 0) <= 512, (n, v)
            assert v.get("scratch", 0) <= (512 if v.get("calls", 0) else 0), (n, v)
            continue
        limit = 20 if "lv_insert" in n else 0
        assert v.get("scratch_ops", 0) == 0, (n, v)
        assert v.get("scratch", 0) <= limit, (n, v)
        assert v.get("vgpr", 0) <= 256, (n, v)
    # the functions those kernels call (an exact check, not a
    # distance heuristic): every scratch instruction is a callee-saved
    # register save or an argument read in the prologue, or a restore in the
    # epilogue; none in a function's body (so none in the solo round loop,
    # which until round 6 read two staging pointers of its argument from
    # scratch, indexed by round parity)
    fns = {n: f for n, f in md.get("functions", {}).items() if "lv_solo" in n}
    assert any("lv_solo_wave" in n for n in fns), sorted(md.get("functions", {}))[:20]
    for n, f in fns.items():
        assert f["frame_violations"] == [], (n, f["frame_violations"][:8])
