"""ISA check of the counted vector-memory waits in the gfx950 code object.

Several kernels of nw_kernels.hip issue a load as inline asm and wait for it
later with a hand-counted `s_waitcnt vmcnt(N)` (the row fill's boundary
prefetch, nw_fill_rows_kernel; the walkers' LDS-DMA windows).  The compiler
does not know about those loads, so two things can break them silently:

  1. the count: fewer than N vector-memory (VMEM) instructions issued between
     the load and the wait on some path -> the wait returns before the load's
     data has landed (GFX9 VMEM ops retire in issue order for vmcnt);
  2. the registers: the compiler sees the asm output as defined at the asm
     statement, so it may copy, read or reuse the destination VGPRs before the
     counted wait (a read sees the old contents, a write is overwritten when
     the load lands).

This walks the disassembly of the code object that was linked into
libsaln.so (build/nw_kernels.o's gfx950 bundle), follows every path from each
VMEM load over the kernel's branches up to the first wait that retires it,
and reports, per load: the waits reached with the VMEM count issued in
between, every instruction on those paths that touches the load's
destination registers, and paths that reach s_endpgm with the load in
flight.  tests/test_isa_handoff.py asserts the row fill's invariants with it.

    python tools/isa_check.py [kernel-substring]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
from dataclasses import dataclass, field

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
OBJ = os.path.join(ROOT, "sequencealigning_amd", "build", "nw_kernels.o")

_VREG = re.compile(r"(?<![\w\[])v\[(\d+):(\d+)\]|(?<![\w\[])v(\d+)\b")
_LINE = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-Fa-f]+):(.*)$")
_TARGET = re.compile(r"<(\S+)\+0x([0-9a-f]+)>")
_FUNC = re.compile(r"^([0-9a-f]+) <(\S+)>:$")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")


@dataclass
class Insn:
    addr: int
    op: str
    args: str
    target: int | None = None  # branch target address

    @property
    def vregs(self) -> set[int]:
        out: set[int] = set()
        for m in _VREG.finditer(self.args.split("//")[0]):
            if m.group(3) is not None:
                out.add(int(m.group(3)))
            else:
                out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        return out

    @property
    def is_vmem(self) -> bool:
        return self.op.startswith(("global_", "buffer_", "flat_", "scratch_"))

    @property
    def is_load(self) -> bool:
        return self.is_vmem and "_load" in self.op and "_lds" not in self.op \
            and not self.op.startswith(("global_atomic", "buffer_atomic", "flat_atomic"))

    def vmcnt(self) -> int | None:
        if self.op != "s_waitcnt":
            return None
        m = _VMCNT.search(self.args)
        return int(m.group(1)) if m else None


@dataclass
class LoadReport:
    insn: Insn
    dest: set[int]
    waits: set[tuple[int, int, int]] = field(default_factory=set)  # (wait addr, N, VMEM count)
    clobbers: set[tuple[int, str]] = field(default_factory=set)    # (addr, op) touching dest
    unwaited_exit: bool = False


def code_object(obj: str = OBJ, out_dir: str = "/tmp") -> str:
    """The gfx950 code object inside a hipcc object file's offload bundle."""
    # per process: parallel test workers must not overwrite each other's files
    fat = os.path.join(out_dir, f"saln_isa_check.{os.getpid()}.fatbin")
    co = os.path.join(out_dir, f"saln_isa_check.{os.getpid()}.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, "/dev/null"],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}",
                    f"--output={co}", "--unbundle"], check=True, capture_output=True)
    return co


def disassemble(co: str) -> dict[str, list[Insn]]:
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout
    funcs: dict[str, list[Insn]] = {}
    cur: list[Insn] | None = None
    base = 0
    for line in txt.splitlines():
        m = _FUNC.match(line)
        if m:
            base = int(m.group(1), 16)
            cur = funcs.setdefault(m.group(2), [])
            continue
        if cur is None:
            continue
        m = _LINE.match(line)
        if not m:
            continue
        ins = Insn(int(m.group(3), 16), m.group(1), m.group(2).strip())
        if ins.op.startswith(("s_branch", "s_cbranch")):
            t = _TARGET.search(m.group(4))
            if t:
                ins.target = base + int(t.group(2), 16)
        cur.append(ins)
    return funcs


def check_function(insns: list[Insn], pick=lambda i: i.is_load, max_count: int = 96):
    """Reports for every VMEM load `pick` selects in one function."""
    at = {ins.addr: k for k, ins in enumerate(insns)}
    reports = []
    for k0, ld in enumerate(insns):
        if not pick(ld):
            continue
        dest = Insn(0, "", ld.args.split(",")[0]).vregs  # the first operand
        rep = LoadReport(ld, dest)
        seen: set[tuple[int, int]] = set()
        stack = [(k0 + 1, 0)]
        while stack:
            k, cnt = stack.pop()
            while True:
                if k >= len(insns) or (k, cnt) in seen or cnt > max_count:
                    break
                seen.add((k, cnt))
                ins = insns[k]
                n = ins.vmcnt()
                if n is not None and cnt >= n:
                    rep.waits.add((ins.addr, n, cnt))
                    break
                if ins.op == "s_endpgm":
                    rep.unwaited_exit = True
                    break
                if ins.vregs & dest:
                    rep.clobbers.add((ins.addr, f"{ins.op} {ins.args}"))
                if ins.is_vmem:
                    cnt += 1
                if ins.op.startswith("s_cbranch") and ins.target is not None:
                    stack.append((at[ins.target], cnt))
                    k += 1
                    continue
                if ins.op == "s_branch" and ins.target is not None:
                    k = at[ins.target]
                    continue
                k += 1
        reports.append(rep)
    return reports


def load_functions(obj: str = OBJ) -> dict[str, list[Insn]]:
    return disassemble(code_object(obj))


def main() -> None:
    sub = sys.argv[1] if len(sys.argv) > 1 else "nw_fill_rows_kernel"
    funcs = load_functions()
    for name, insns in funcs.items():
        if sub not in name:
            continue
        print(name)
        for r in check_function(insns):
            waits = sorted({(n, c) for _, n, c in r.waits})
            flag = ("  CLOBBER" if r.clobbers else "") + ("  IN-FLIGHT-AT-EXIT" if r.unwaited_exit else "")
            print(f"  {r.insn.addr:#x} {r.insn.op} {r.insn.args}: waits (N, count) {waits}{flag}")
            for a, s in sorted(r.clobbers)[:4]:
                print(f"      {a:#x} {s}")


if __name__ == "__main__":
    main()
