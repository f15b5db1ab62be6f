"""Static check of the gfx950 MFMA data hazards in the built library.

hipcc pads the wait states between an MFMA and the instructions around it only for instructions it
generated itself. An inline-asm statement is opaque to its hazard recognizer (it pads one state after
the statement, nothing inside it), so an asm VALU instruction that reads an MFMA result too early,
or writes an MFMA operand too late, returns stale data on some waves of some launches -- no fault,
no message (round 3: an asm `v_pk_max_f16` on the MFMA accumulator failed 76 GPU tests with garbage
and run-to-run differences). This scanner re-derives the two rules from the disassembly of every
kernel and flags every site that violates them, whoever generated it:

  R1  MFMA writes VGPR/AGPR d  ->  any non-MFMA instruction reads or writes d:
      >= MFMA_WRITE_STATES[opcode] wait states in between (XDL write -> VALU/VMEM/LDS access)
  R2  VALU writes VGPR v  ->  an MFMA reads v as SrcA or SrcB: >= 2 wait states
      (LLVM GCNHazardRecognizer "LegacyVALUNotDotWritesVGPRWaitStates" for gfx940/gfx950)

A wait state is one issued instruction; `s_nop N` counts N + 1. An MFMA that reads its own
destination as SrcC (the accumulation chain) is exempt from R1. The analysis follows the control
flow: basic blocks from the branch targets, entry states merged over every predecessor (the
smallest distance since the producer wins), iterated to a fixed point, so a producer before a loop's
back edge is checked against the consumers at the loop head. Calls and indirect jumps end the path
(callees start with nothing pending; the compiler pads the call boundary itself).

The thresholds were checked against the compiler's own schedule for the one MFMA this library uses
(v_mfma_f32_16x16x32_f16, 4 passes on gfx950): hipcc's own consumers sit at >= 8 states after the
MFMA (5,972 of them at exactly 8) and its own VALU producers at >= 2 states before an MFMA source
operand -- so a clean compiler build scans clean and any shorter distance is an asm site.

  python tools/hazard_scan.py [lib/libtcnn_mi355x.so]     (prints every violation)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# XDL write -> non-MFMA access, per opcode (gfx950). Add a row before using a new MFMA shape: an
# unknown opcode is reported as a violation rather than assumed safe.
MFMA_WRITE_STATES = {
    "v_mfma_f32_16x16x32_f16": 8,   # 4-pass
    "v_mfma_f32_16x16x32_bf16": 8,  # 4-pass
    "v_mfma_f32_32x32x16_f16": 16,  # 8-pass (12 on gfx950 per the guide; 16 is conservative)
    "v_mfma_f32_32x32x16_bf16": 16,
}
VALU_TO_MFMA_SRC_AB = 2
# A taken branch is followed by an instruction-fetch bubble before the target issues; it counts one
# state beyond the branch instruction itself. hipcc's own schedule relies on this: its only MFMA ->
# VALU distances below 8 on this library (21 sites, all of them 7) are paths through a taken branch.
TAKEN_BRANCH_EXTRA = 1
CAP = 32  # distances beyond this never matter

_REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")
_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_NOT_VDST = ("v_cmp", "v_cmpx", "v_readlane", "v_readfirstlane", "v_mfma")
_END = ("s_endpgm", "s_setpc_b64", "s_trap")
_CALL = ("s_swappc_b64", "s_call_b64")


def regs(text):
    out = set()
    for m in _REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            for r in range(int(m.group(4)), int(m.group(5)) + 1):
                out.add((m.group(3), r))
    return out


def _split_ops(ops):
    # operands are comma separated at the top level; register ranges contain ':' not ','
    return [p.strip() for p in ops.split(",")] if ops.strip() else []


def code_objects(lib, workdir):
    """Yield the disassembly text of every gfx950 code object in the library's .hip_fatbin."""
    fat = os.path.join(workdir, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(workdir, "stripped")],
                   check=True)
    b = open(fat, "rb").read()
    offs = []
    i = b.find(MAGIC)
    while i >= 0:
        offs.append(i)
        i = b.find(MAGIC, i + 1)
    for k, o in enumerate(offs):
        part, co = os.path.join(workdir, f"p{k}"), os.path.join(workdir, f"p{k}.co")
        open(part, "wb").write(b[o:offs[k + 1] if k + 1 < len(offs) else len(b)])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        yield subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                             text=True).stdout


def disassemble_object(path):
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", path], check=True, capture_output=True,
                          text=True).stdout


def functions(dis):
    """Split a disassembly into (name, [(addr, mnemonic, ops, text)]) for the functions that issue MFMAs
    (the others cannot violate R1/R2 and are skipped unparsed)."""
    chunks = dis.split(">:\n")
    for k in range(len(chunks) - 1):
        name = chunks[k].rsplit("<", 1)[1]
        text = chunks[k + 1]
        if "v_mfma" not in text:
            continue
        body = []
        for line in text.split("\n"):
            if not line.startswith("\t"):
                if line.endswith(">") or line.startswith("0"):
                    break  # the next function's header line
                continue
            code, _, comment = line.partition("//")
            ins = code.strip()
            m = _ADDR.search("//" + comment)
            if not ins or not m:
                continue
            mn, _, ops = ins.partition(" ")
            body.append((int(m.group(1), 16), mn, ops, ins))
        yield name, body


class _Ins:
    __slots__ = ("addr", "mn", "text", "ws", "mfma", "wstates", "dst", "touch", "srcab", "srcc", "valu_dst", "target",
                 "cond", "end", "call")


def _decode(addr, mn, ops, text):
    i = _Ins()
    i.addr, i.mn, i.text = addr, mn, text
    parts = _split_ops(ops)
    i.ws = int(parts[0], 0) + 1 if mn == "s_nop" else 1
    i.mfma = mn.startswith("v_mfma")
    i.wstates = MFMA_WRITE_STATES.get(mn.split("_e64")[0]) if i.mfma else None
    i.touch = regs(ops)
    i.dst = regs(parts[0]) if i.mfma and parts else set()
    i.srcab = (regs(parts[1]) | regs(parts[2])) if i.mfma and len(parts) > 2 else set()
    i.srcc = regs(parts[3]) if i.mfma and len(parts) > 3 else set()
    i.valu_dst = set()
    if mn.startswith("v_") and not mn.startswith(_NOT_VDST) and parts:
        i.valu_dst = {r for r in regs(parts[0]) if r[0] == "v"}
    i.target, i.cond, i.end, i.call = None, False, False, mn in _CALL
    if mn == "s_branch" or mn.startswith("s_cbranch"):
        i.target = addr + 4 + 4 * int(parts[0], 0)
        i.cond = mn != "s_branch"
    elif mn in _END:
        i.end = True
    return i


def _merge(a, b):
    """Entry state of a block reached from two paths: per register the closest producer."""
    if a is None:
        return dict(b)
    out = dict(a)
    for k, v in b.items():
        if k not in out or v[0] < out[k][0]:
            out[k] = v
    return out


def check_function(body):
    """Return the violations of R1/R2 in one function: [(consumer text, producer text, states, rule)]."""
    ins = [_decode(*x) for x in body]
    if not any(i.mfma for i in ins):
        return []
    index = {i.addr: k for k, i in enumerate(ins)}
    leaders = {0}
    for k, i in enumerate(ins):
        if i.target is not None or i.end or i.call:
            if k + 1 < len(ins):
                leaders.add(k + 1)
            if i.target in index:
                leaders.add(index[i.target])
    starts = sorted(leaders)
    blocks = {s: (starts[j + 1] if j + 1 < len(starts) else len(ins)) for j, s in enumerate(starts)}
    # state: (kind, reg) -> (states since the producer, producer index); kind 'm' = MFMA dst, 'v' = VALU dst
    entry = {0: {}}
    violations = {}

    def run(s, state, record):
        st = dict(state)
        for k in range(s, blocks[s]):
            i = ins[k]
            for (kind, r), (el, p) in list(st.items()):
                if kind == "m" and r in i.touch and not i.mfma:
                    need = ins[p].wstates
                    if need is None or el < need:
                        record((k, p, "R1", el))
                elif kind == "v" and i.mfma and r in i.srcab and el < VALU_TO_MFMA_SRC_AB:
                    record((k, p, "R2", el))
            # the instruction's own writes replace older producers of the same registers
            if i.mfma:
                for r in i.dst:
                    st[("m", r)] = (0, k)
                    st.pop(("v", r), None)
            if i.valu_dst:
                for r in i.valu_dst:
                    st[("v", r)] = (0, k)
                    st.pop(("m", r), None)
            # advance: every pending producer except this instruction's own gets this instruction's states
            nxt = {}
            for key, (el, p) in st.items():
                if p != k:
                    el += i.ws
                if key[0] == "m" and el >= (ins[p].wstates or CAP):
                    continue
                if key[0] == "v" and el >= VALU_TO_MFMA_SRC_AB:
                    continue
                nxt[key] = (el, p)
            st = nxt
            if i.call:
                # the callee starts clean and the compiler pads the call boundary: resume with nothing pending
                return ([(k + 1, {})] if k + 1 < len(ins) else [])
            succ = []
            if i.target is not None and i.target in index:
                succ.append((index[i.target], _advance(st, TAKEN_BRANCH_EXTRA)))
            if i.end or (i.target is not None and not i.cond):
                return succ
            if k + 1 == blocks[s] and k + 1 < len(ins):
                succ.append((k + 1, st))
                return succ
        return []

    def _advance(st, n):
        out = {}
        for key, (el, p) in st.items():
            el += n
            if key[0] == "m" and el >= (ins[p].wstates or CAP):
                continue
            if key[0] == "v" and el >= VALU_TO_MFMA_SRC_AB:
                continue
            out[key] = (el, p)
        return out

    work = [0]
    while work:
        s = work.pop()
        for t, out in run(s, entry[s], lambda v: None):
            new = _merge(entry.get(t), out)
            if entry.get(t) != new:
                entry[t] = new
                work.append(t)
    for s in blocks:
        # a block no analysed path reaches (an indirect target) starts with nothing pending
        run(s, entry.get(s, {}), lambda v: violations.setdefault((v[0], v[1], v[2]), v[3]))
    return [(ins[c].text, ins[p].text, el, rule) for (c, p, rule), el in sorted(violations.items())]


def scan_disassembly(dis):
    out = {}
    for name, body in functions(dis):
        v = check_function(body)
        if v:
            out[name] = v
    return out


def scan(lib):
    hits, n = {}, 0
    with tempfile.TemporaryDirectory() as d:
        for dis in code_objects(lib, d):
            n += 1
            hits.update(scan_disassembly(dis))
    return hits, n


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                              "neuralbtf-tiny-cuda-nn_amd", "lib", "libtcnn_mi355x.so")
    if lib.endswith(".o"):
        hits, n = scan_disassembly(disassemble_object(lib)), 1
    else:
        hits, n = scan(lib)
    print(f"{n} code objects scanned, {sum(len(v) for v in hits.values())} violations in {len(hits)} kernels")
    for k, v in hits.items():
        print(len(v), k)
        for c in v[:4]:
            print("    ", c)
