"""Static instruction mix of the kernels in a hipcc -save-temps assembly file.

    python tools/isa_count.py path/to/x-hip-amdgcn-amd-amdhsa-gfx950.s [substring ...]

Prints, per kernel whose symbol contains every substring: VALU / SALU / VMEM / LDS (ds_) / DPP instruction counts of
the straight-line text (loops are not unrolled further: a static count, not an executed count) and the
.vgpr_count / .sgpr_count / spill fields of the kernel descriptor metadata.
"""
import re
import sys


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    s = open(path).read()
    meta = s[s.find("amdhsa.kernels"):]
    for m in re.finditer(r"^(_Z\w+):\s*;", s, re.M):
        name = m.group(1)
        if not all(x in name for x in subs):
            continue
        body = s[m.end():s.find(".Lfunc_end", m.end())]
        ins = [l.strip() for l in body.split("\n")]
        ins = [l for l in ins if l and not l.startswith((".", ";")) and not l.endswith(":")]
        cnt = {
            "valu": sum(l.startswith("v_") for l in ins),
            "dpp": sum(l.startswith("v_") and "_dpp" in l.split()[0] for l in ins),
            "salu": sum(l.startswith("s_") and not l.startswith(("s_waitcnt", "s_barrier", "s_nop")) for l in ins),
            "vmem": sum(l.startswith(("global_", "buffer_", "flat_")) for l in ins),
            "lds": sum(l.startswith("ds_") for l in ins),
            "waitcnt": sum(l.startswith("s_waitcnt") for l in ins),
        }
        k = meta.find(".name:           " + name)
        # the descriptor entry around ".name": from the entry's start ("  - ." line) to the next entry
        st = meta.rfind("\n  - .", 0, k) if k >= 0 else -1
        en = meta.find("\n  - .", k) if k >= 0 else -1
        blk = meta[st:en if en > 0 else len(meta)] if k >= 0 else ""
        regs = {f: (re.search(r"\." + f + r":\s+(\d+)", blk) or [None, "?"])[1]
                for f in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count")}
        print(name[:90])
        print("   ", " ".join(f"{k}={v}" for k, v in cnt.items()), "|", " ".join(f"{k}={v}" for k, v in regs.items()))


if __name__ == "__main__":
    main()
