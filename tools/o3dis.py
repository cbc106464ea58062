"""Disassemble an O3-tier code object into text the CPU simulator (tests/asmsim) runs.

The O3 tier's kernels are compiled by LLVM (comgr) from the specialised HIP source; to count
their instructions per candidate, model their LDS bank conflicts and check their verdicts on the
CPU, the simulator runs their machine code.  llvm-objdump prints branches as word offsets with the
target in a comment; this turns every target into a label and adds the kernel's LDS size.

  python tools/o3dis.py <code object> [out.s]

Also importable: ``convert(co_path) -> str``.  Test / measurement infrastructure only."""
import re
import subprocess
import sys
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
_KSYM = re.compile(r"^([0-9a-fA-F]+) <([^>]+)>:$")
_TGT = re.compile(r"<([A-Za-z_.$][\w.$]*)\+0x([0-9a-fA-F]+)>")
_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_BRANCH = ("s_cbranch_", "s_branch")
_SKIP = ("s_code_end",)


def _lds_sizes(co: str) -> dict:
    notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", co], capture_output=True, text=True,
                           check=True).stdout
    sizes, cur = {}, None
    for ln in notes.splitlines():
        m = re.match(r"^    \.group_segment_fixed_size:\s+(\d+)", ln)
        if m:
            cur = int(m.group(1))
        m = re.match(r"^    \.name:\s+(\S+)", ln)
        if m and cur is not None:
            sizes[m.group(1)] = cur
            cur = None
    return sizes


_LINE = re.compile(r"^; \S+\.hip:(\d+)$")


def _image(co: str) -> bytes:
    """the code object's PT_LOAD segments at their virtual addresses (vaddr 0 up)"""
    import struct
    b = Path(co).read_bytes()
    if b[:4] != b"\x7fELF" or b[4] != 2:
        raise ValueError("not an ELF64 code object: " + co)
    phoff, = struct.unpack_from("<Q", b, 0x20)
    phentsize, phnum = struct.unpack_from("<HH", b, 0x36)
    segs = []
    for i in range(phnum):
        ptype, _flags, off, vaddr, _paddr, filesz, memsz, _align = struct.unpack_from("<IIQQQQQQ", b, phoff + i * phentsize)
        if ptype == 1:  # PT_LOAD
            segs.append((vaddr, b[off:off + filesz], memsz))
    img = bytearray(max((v + m for v, _, m in segs), default=0))
    for v, data, _ in segs:
        img[v:v + len(data)] = data
    return bytes(img)


def convert(co: str, lines: bool = False, image: str = None) -> str:
    """``lines``: a code object built with -gline-tables-only (MYTHGPU_JIT_EXTRA) — every
    instruction is tagged with its source line ("; vcode line N"), so the simulator's per-tag
    counts (ASMSIM_COUNT) attribute the O3 kernel's VALU to the statements of its source."""
    dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950"] + (["-l"] if lines else []) + [co],
                         capture_output=True, text=True, check=True).stdout
    sizes = _lds_sizes(co)
    base = {}
    insts = []  # (address, text, target or None) / ("kernel", name)
    for ln in dis.splitlines():
        lm = _LINE.match(ln.strip())
        if lm:
            insts.append(("line", lm.group(1)))
            continue
        m = _KSYM.match(ln.strip())
        if m:
            base[m.group(2)] = int(m.group(1), 16)
            insts.append(("kernel", m.group(2)))
            continue
        if not ln.startswith("\t"):
            continue
        body, _, comment = ln.partition("//")
        text = body.strip()
        if not text or text.startswith(_SKIP):
            continue
        am = _ADDR.search("//" + comment)
        addr = int(am.group(1), 16) if am else None
        tgt = None
        if text.startswith(_BRANCH):
            tm = _TGT.search(comment)
            if not tm:
                raise ValueError("branch without a target: " + ln)
            tgt = base[tm.group(1)] + int(tm.group(2), 16)
            text = text.split()[0] + " L%x" % tgt
        insts.append((addr, text, tgt))
    targets = {t for i in insts if i[0] not in ("kernel", "line") for t in [i[2]] if t is not None}
    out = []
    if any(i[0] not in ("kernel", "line") and i[1].startswith("s_getpc_b64") for i in insts):
        # PC-relative reads of the code object's own data (baked tables): the simulator maps its image
        image = image or co + ".img"
        Path(image).write_bytes(_image(co))
        out.append(".asmsim_image " + str(Path(image).resolve()))
    for name, size in sizes.items():
        out += [".amdhsa_kernel " + name, ".amdhsa_group_segment_fixed_size %d" % size, ".end_amdhsa_kernel"]
    for i in insts:
        if i[0] == "kernel":
            out.append(i[1] + ":")
            continue
        if i[0] == "line":
            out.append("  ; vcode line " + i[1])
            continue
        addr, text, _ = i
        if addr in targets:
            out.append("L%x:" % addr)
        if text.startswith("s_getpc_b64"):
            out.append(".asmsim_pc 0x%x" % addr)
        out.append("  " + text)
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    s = convert(sys.argv[1], lines="-l" in sys.argv)
    sys.argv = [a for a in sys.argv if a != "-l"]
    if len(sys.argv) > 2:
        Path(sys.argv[2]).write_text(s)
    else:
        sys.stdout.write(s)
