"""Per-kernel register / spill / LDS report for one HIP source, built for gfx950 on the host.

    python scripts/tools/kernel_regs.py lumen/csrc/kernels/flash_attn.hip [name-filter]

Compiles the device side only (``--cuda-device-only -S``) and reads the kernel descriptors the
assembler emits (.vgpr_count / .agpr_count / .private_segment_fixed_size / .group_segment...),
plus the number of scratch instructions in each kernel body, so a change that pushes a hot
kernel over its launch-bounds register budget shows up before any GPU run."""
import os
import re
import subprocess
import sys
import tempfile

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def report(src, filt=""):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run([os.path.join(ROCM, "bin", "hipcc"), "--offload-arch=gfx950", "-O3",
                        "-std=c++17", "-w", "--cuda-device-only", "-S", src, "-o", out], check=True)
        s = open(out).read()
    rows = []
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        name = m.group(1)
        if filt and filt not in name:
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]
        scratch = len(re.findall(r"\bscratch_(load|store)", body))
        # the compiler's per-function summary comments follow .Lfunc_end
        tail = s[end:s.find(".end_amdhsa_kernel", end) if ".end_amdhsa_kernel" in s[end:] else end + 4000]

        def field(key):
            f = re.search(rf"; {key}: (\d+)", tail)
            return int(f.group(1)) if f else -1
        rows.append((name, field("NumVgprs"), field("NumAgprs"), field("ScratchSize"), scratch,
                     field("LDSByteSize"), field("Occupancy")))
    for n, v, a, p, sc, lds, occ in rows:
        flag = "  SPILL" if p or sc else ""
        print(f"vgpr {v:4d} agpr {a:4d} occ {occ} scratch {p:4d} B / {sc:3d} ops lds {lds:6d}  "
              f"{n[:90]}{flag}")


if __name__ == "__main__":
    report(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
