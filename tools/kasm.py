"""Dump one kernel's gfx950 assembly from csrc/packed_codec.hip (device-only
compile) and print instruction statistics.  Usage:
  python tools/kasm.py sp_encode_kernelILb0 [-DCPK_SP_WPE=2 ...] [--out /tmp/k.s]"""
import collections
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
SRC = REPO / "capnproto-java_amd" / "csrc" / "packed_codec.hip"


def main():
    name = sys.argv[1]
    flags = [a for a in sys.argv[2:] if a.startswith("-D")]
    out = "/tmp/kasm_full.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-S",
                    "--cuda-device-only", "-Wno-unused-value", "-Wno-unused-result", *flags,
                    str(SRC), "-o", out], check=True)
    s = open(out).read()
    m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):", s, re.M)
    i = m.start()
    j = s.index(".Lfunc_end", i)
    body = [l for l in s[i:j].split("\n") if l.startswith("\t") and not l.strip().startswith((";", "."))]
    Path("/tmp/kasm_kernel.s").write_text("\n".join(body))
    ops = collections.Counter(l.split()[0] for l in body)
    print(m.group(1), "instructions:", len(body))
    salu = sum(v for k, v in ops.items() if k.startswith("s_"))
    valu = sum(v for k, v in ops.items() if k.startswith("v_"))
    print("SALU", salu, "VALU", valu, "DS", sum(v for k, v in ops.items() if k.startswith("ds_")))
    print(ops.most_common(30))


if __name__ == "__main__":
    main()
