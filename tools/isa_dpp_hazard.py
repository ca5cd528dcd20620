"""Check the gfx950 code objects of libgpk.so for the DPP read hazard that inline asm hides from the compiler:
a VALU write of a VGPR needs two wait states before a DPP instruction reads that VGPR as its DPP source (src0).
Disassembles every gfx950 code object of the library (llvm-objdump --offloading, in a scratch directory) and
walks back from each DPP instruction over the preceding instructions of its block.

usage: python tools/isa_dpp_hazard.py [libgpk.so]   (exit status 1 and a listing if any hazard is found)"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def regs(tok):
    """Register numbers of a v operand: v7 -> {7}, v[4:5] -> {4, 5}."""
    tok = tok.strip().lstrip("-|").rstrip("|")
    m = re.match(r"v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def wait_states(mn, ops):
    if mn == "s_nop":
        return int(ops[0], 0) + 1 if ops else 1
    return 1


def check_lines(lines):
    """lines: disassembly lines of one code object -> list of (dpp line, writer line)."""
    insts = []
    for ln in lines:
        s = ln.split("//")[0].strip()
        if not s:
            continue
        if s.endswith(">:") or s.endswith(":"):
            insts.append(("<label>", [], ln))
            continue
        parts = s.split(None, 1)
        mn = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        insts.append((mn, ops, ln))
    bad = []
    for i, (mn, ops, ln) in enumerate(insts):
        if not mn.endswith("_dpp") or len(ops) < 2:
            continue
        src = regs(ops[1].split()[0])
        ws = 0
        for j in range(i - 1, -1, -1):
            pm, pops, pln = insts[j]
            if pm == "<label>" or pm.startswith("s_cbranch") or pm.startswith("s_branch"):
                bad.append((ln.strip(), "block boundary within two wait states"))
                break
            if pm.startswith("v_") and pops and not pm.startswith("v_readlane") and not pm.startswith("v_cmp"):
                if regs(pops[0]) & src:
                    bad.append((ln.strip(), pln.strip()))
                    break
            ws += wait_states(pm, pops)
            if ws >= 2:
                break
    return bad


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..",
                                                              "gaussianprocessfundamentals_amd", "libgpk.so")
    tmp = tempfile.mkdtemp()
    try:
        shutil.copy(lib, os.path.join(tmp, "lib.so"))
        subprocess.run([OBJDUMP, "--offloading", "lib.so"], cwd=tmp, check=True, capture_output=True)
        n_dpp, bad = 0, []
        for f in sorted(os.listdir(tmp)):
            if not f.endswith("gfx950"):
                continue
            out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", os.path.join(tmp, f)], check=True,
                                 capture_output=True, text=True).stdout.splitlines()
            n_dpp += sum(1 for ln in out if "_dpp " in ln)
            bad += check_lines(out)
        print("DPP instructions: %d, hazards: %d" % (n_dpp, len(bad)))
        for d, w in bad[:20]:
            print("  %s\n    after: %s" % (d, w))
        return 1 if bad else 0
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
