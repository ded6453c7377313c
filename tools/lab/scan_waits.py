"""Lab (CPU): find kernels whose global loads are serialised -- a load
followed by a full `s_waitcnt vmcnt(0)` before the next one (typically a
guarded load `i < n ? x[i] : 0` compiled to a branch and a wait per element).

    python tools/lab/scan_waits.py [csrc files ...]

Compiles each source to gfx950 assembly with the product's flags and lists
every kernel with at least 4 loads of which at least half are followed
directly by a full wait."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from text_guided_face_recognition_amd import build as B  # noqa: E402


def scan(src, tmp):
    asm = os.path.join(tmp, os.path.basename(src) + ".s")
    flags = B.FILE_FLAGS.get(os.path.basename(src), [])
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", *flags,
                    "--cuda-device-only", "-S", "-I", B.CSRC, src, "-o", asm],
                   check=True, capture_output=True)
    s = open(asm).read()
    for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
        body = s[m.end():s.find(".Lfunc_end", m.end())]
        seq = []
        for line in body.split("\n"):
            line = line.strip()
            if line.startswith(("global_load", "buffer_load")):
                seq.append("L")
            elif line.startswith("s_waitcnt") and "vmcnt(0)" in line:
                seq.append("W")
        serial = sum(1 for a, b in zip(seq, seq[1:]) if a == "L" and b == "W")
        loads = seq.count("L")
        if loads >= 4 and serial >= 0.5 * loads:
            print(f"{os.path.basename(src)}: {m.group(1)[:80]}  loads {loads}  "
                  f"load->vmcnt(0) {serial}")


def main(files):
    files = files or [os.path.join(B.CSRC, f) for f in sorted(os.listdir(B.CSRC))
                      if f.endswith(".hip")]
    with tempfile.TemporaryDirectory() as tmp:
        for f in files:
            scan(f, tmp)


if __name__ == "__main__":
    main(sys.argv[1:])
