"""Register / scratch usage of every kernel in a hipcc object (gfx950 code object metadata).

    python tools/kernel_resources.py cosnet_amd/_lib/obj/gemm.o [name-substring]

Prints kernels with their VGPR / AGPR / SGPR counts, spill counts and private-segment (scratch)
size; exits non-zero if any kernel uses scratch (the check every build's ISA must pass)."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main(obj, flt=""):
    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "k.co")
        fb = os.path.join(d, "fb.bin")
        # the device code sits in the object's .hip_fatbin section as an offload bundle
        subprocess.run([LLVM + "/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb],
                       check=True)
        subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + fb,
                        "--output=" + co], check=True)
        notes = subprocess.run([LLVM + "/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    ks = re.split(r"\n\s+- \.agpr_count:", notes)
    bad = 0
    rows = []
    for k in ks[1:]:
        get = lambda key: (re.search(r"\." + key + r":\s+(\S+)", k) or [None, "?"])[1]
        name = get("name")
        if flt and flt not in name:
            continue
        agpr = k.split("\n")[0].strip()
        scratch = int(get("private_segment_fixed_size"))
        rows.append((name, get("vgpr_count"), agpr, get("sgpr_count"), get("vgpr_spill_count"),
                     get("sgpr_spill_count"), scratch))
        bad += scratch > 0
    for r in rows:
        print("%-100s vgpr %4s agpr %4s sgpr %4s spill v%s s%s scratch %d" % ((r[0][:100],) + r[1:]))
    print("%d kernels, %d with scratch" % (len(rows), bad))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""))
