"""ISA check of the EI kernel's asm-load ring (test infrastructure).

``gp_score_kernel`` streams its B fragments through ``global_load_dwordx2``
issued from inline asm with an ``"=v"`` output and explicit ``s_waitcnt vmcnt``
ties (mpi_opt_amd/csrc/gp.hip, MPO_LD / MPO_EI_GROUP).  The compiler believes
such a destination is written when the load issues, so nothing in the source
stops it from reading, copying or reusing that register before the matching
wait -- a hazard only the generated code can rule out.

This module extracts the gfx950 code objects from libmpo.so's
``.hip_fatbin`` offload bundles, disassembles them with llvm-objdump and runs a
dataflow over each kernel's control-flow graph: the state is the ordered list of
outstanding vector-memory operations (their destination VGPRs); ``s_waitcnt
vmcnt(k)`` retires the oldest until k remain (gfx9 vector memory returns in
issue order); any other instruction that names a VGPR still owed by an
outstanding load is a hazard, and so is a call with loads outstanding.
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_VMEM = ("global_", "buffer_", "flat_", "scratch_")
_REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
_INSN = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_TARGET = re.compile(r"<(.+?)\+0x([0-9a-f]+)>")


def gfx950_code_objects(lib_path):
    """The gfx950 ELF code objects inside ``lib_path``'s offload bundles."""
    data = open(lib_path, "rb").read()
    out = []
    pos = data.find(_MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if triple.endswith("gfx950") and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(_MAGIC, pos + 1)
    return out


def disassemble(code_object):
    with tempfile.TemporaryDirectory() as tmp:
        fn = os.path.join(tmp, "co.o")
        with open(fn, "wb") as fh:
            fh.write(code_object)
        return subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", fn], check=True, capture_output=True,
                              text=True).stdout


def functions(text):
    """{name: [(addr, mnemonic, operands, target_addr|None)]} of a disassembly."""
    funcs, cur, base = {}, None, {}
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = m.group(2)
            base[cur] = int(m.group(1), 16)
            funcs[cur] = []
            continue
        m = _INSN.match(line)
        if m and cur is not None:
            mn, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
            tgt = None
            if mn.startswith("s_branch") or mn.startswith("s_cbranch"):
                t = _TARGET.search(line)
                if t:
                    tgt = ("sym", t.group(1), int(t.group(2), 16))
            funcs[cur].append([addr, mn, ops, tgt])
    for name, insns in funcs.items():
        for ins in insns:
            if ins[3] is not None:
                _, sym, off = ins[3]
                ins[3] = base.get(sym, base[name]) + off
    return funcs


def vregs(ops):
    out = set()
    for m in _REG.finditer(ops):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _split_first(ops):
    depth, i = 0, 0
    for i, ch in enumerate(ops):
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        elif ch == "," and depth == 0:
            return ops[:i], ops[i + 1:]
    return ops, ""


def _vmem_effect(mn, ops):
    """(destination VGPRs, VGPRs read) of a vector-memory instruction."""
    first, rest = _split_first(ops)
    returns = ("_load" in mn and "_lds" not in mn and " lds" not in " " + ops) or \
              ("atomic" in mn and re.search(r"\b(glc|sc0)\b", ops) is not None)
    if returns:
        return vregs(first), vregs(rest)
    return set(), vregs(ops)


def _vmcnt(ops):
    m = re.search(r"vmcnt\((\d+)\)", ops)
    return int(m.group(1)) if m else None


_SREG = re.compile(r"^\s*(?:s(\d+)|s\[(\d+):(\d+)\]|(vcc))(?!\w)")


def _sdest(ops):
    """Destination scalar register range of an instruction's first operand (or None)."""
    m = _SREG.match(ops)
    if not m:
        return None
    if m.group(4):
        return ("vcc",)
    if m.group(1) is not None:
        return (int(m.group(1)), int(m.group(1)))
    return (int(m.group(2)), int(m.group(3)))


def _scalar_step(known, mn, ops):
    """Track the few scalar facts that decide ``s_cbranch_vcc*`` in the ring's loop
    exits: ``s_mov_b64 s[a:b], imm`` then ``s_and_b64 vcc, exec, s[a:b]`` (vcc is
    non-zero iff the constant is, exec being non-zero).  Returns the new facts."""
    d = _sdest(ops)
    out = dict(known)
    if mn == "s_mov_b64" and d and d != ("vcc",):
        src = ops.split(",", 1)[1].strip()
        try:
            out = {k: v for k, v in out.items() if k == "vcc" or k[1] < d[0] or k[0] > d[1]}
            out[d] = int(src, 0)
            return out
        except ValueError:
            pass
    if mn == "s_and_b64" and d == ("vcc",):
        parts = [p.strip() for p in ops.split(",")]
        out.pop("vcc", None)
        if len(parts) == 3 and parts[1] == "exec":
            m = re.match(r"s\[(\d+):(\d+)\]$", parts[2])
            if m and (int(m.group(1)), int(m.group(2))) in known:
                out["vcc"] = known[(int(m.group(1)), int(m.group(2)))] != 0
        return out
    if d == ("vcc",) or mn.startswith("v_cmp") or "vcc" in ops.split(",")[0]:
        out.pop("vcc", None)
    if d and d != ("vcc",):
        out = {k: v for k, v in out.items() if k == "vcc" or k[1] < d[0] or k[0] > d[1]}
    return out


def check_function(insns, max_states=64):
    """Hazards [(addr, mnemonic, operands, owed VGPRs)] in one function."""
    if not insns:
        return []
    addrs = [i[0] for i in insns]
    index = {a: k for k, a in enumerate(addrs)}
    leaders = {0}
    for k, (_, mn, _, tgt) in enumerate(insns):
        if tgt is not None and tgt in index:
            leaders.add(index[tgt])
        if mn.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")) and k + 1 < len(insns):
            leaders.add(k + 1)
    starts = sorted(leaders)
    blocks = {s: (s, (starts[j + 1] if j + 1 < len(starts) else len(insns))) for j, s in enumerate(starts)}
    hazards = []
    seen = {}
    work = [(0, (), ())]
    while work:
        b, state, facts = work.pop()
        st = seen.setdefault(b, set())
        if (state, facts) in st or len(st) >= max_states:
            continue
        st.add((state, facts))
        s0, s1 = blocks[b]
        q = list(state)
        known = dict(facts)
        falls = True
        succ = []
        for k in range(s0, s1):
            addr, mn, ops, tgt = insns[k]
            owed = set().union(*q) if q else set()
            if mn in ("s_cbranch_vccnz", "s_cbranch_vccz") and "vcc" in known:
                taken = known["vcc"] if mn == "s_cbranch_vccnz" else not known["vcc"]
                if taken:
                    falls = False
                    if tgt in index:
                        succ.append(index[tgt])
                continue
            if mn.startswith("s_"):
                known = _scalar_step(known, mn, ops)
            elif mn.startswith("v_cmp") or ops.startswith("vcc"):
                known.pop("vcc", None)
            if mn == "s_waitcnt" or mn.startswith("s_waitcnt_vmcnt"):
                n = _vmcnt(ops)
                if n is not None:
                    q = q[max(0, len(q) - n):]
                continue
            if mn.startswith(_VMEM):
                dest, reads = _vmem_effect(mn, ops)
                bad = (reads | dest) & owed
                if bad:
                    hazards.append((addr, mn, ops, sorted(bad)))
                q.append(frozenset(dest))
                continue
            if mn.startswith(("s_swappc", "s_call")) and any(q):
                hazards.append((addr, mn, ops, sorted(owed)))
            bad = vregs(ops) & owed
            if bad:
                hazards.append((addr, mn, ops, sorted(bad)))
            if tgt is not None and tgt in index:
                succ.append(index[tgt])
            if mn.startswith("s_branch") or mn.startswith("s_endpgm") or mn.startswith("s_setpc"):
                falls = False
        if falls and s1 < len(insns):
            succ.append(s1)
        facts = tuple(sorted(known.items(), key=repr))
        for nb in succ:
            work.append((nb, tuple(q), facts))
    return sorted(set((a, m, o, tuple(r)) for a, m, o, r in hazards))


def check_library(lib_path, pattern="gp_score_kernel"):
    """{kernel: hazards} for every function of ``lib_path`` whose name contains ``pattern``."""
    out = {}
    for co in gfx950_code_objects(lib_path):
        for name, insns in functions(disassemble(co)).items():
            if pattern in name:
                out[name] = check_function(insns)
    return out
