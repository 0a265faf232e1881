"""Static instruction mix per loop of a kernel in an amdgcn .s file (diagnostic).
usage: isa_loops.py file.s [kernel-substring]
Counts VALU (v_*), SALU (s_* minus waits/branches), LDS (ds_*), VMEM (global_/buffer_),
waitcnt and barriers in every loop (by LLVM's loop comments), with the 4-cycle ops
(measured issue cost, profiles/r3_valu_issue_rates.txt) counted separately."""
import collections, re, sys

FULL = ("v_add_u32", "v_sub_u32", "v_xor_b32", "v_lshrrev_b32", "v_lshlrev_b32", "v_and_b32",
        "v_or_b32", "v_mov_b32", "v_subrev_u32", "v_add_co_u32", "v_sub_co_u32", "v_not_b32",
        "v_ashrrev_i32", "v_addc_co_u32", "v_subb_co_u32", "v_cndmask_b32")


def kernels(lines, want):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            if cur and want in cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            body.append(ln)
    if cur and want in cur:
        yield cur, body


def main():
    src = open(sys.argv[1]).read().splitlines()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, body in kernels(src, want):
        print("==", name[:80])
        blk_loop = None
        stats = collections.defaultdict(collections.Counter)
        order = []
        for ln in body:
            m = re.match(r"^\.(LBB\w+):(.*)", ln)
            if m:
                c = m.group(2)
                h = re.search(r"Header=(BB\w+) Depth=(\d+)", c)
                if "Loop Header" in c:
                    blk_loop = "L" + m.group(1)[1:] + " d" + re.search(r"Depth=(\d+)", c).group(1)
                elif h:
                    blk_loop = "L" + h.group(1) + " d" + h.group(2)
                else:
                    blk_loop = None
                if blk_loop and blk_loop not in order:
                    order.append(blk_loop)
                continue
            t = ln.strip()
            if not t or t.startswith((";", ".")):
                continue
            op = t.split()[0]
            key = blk_loop or "straight"
            st = stats[key]
            if op.startswith("v_"):
                st["valu"] += 1
                if not op.startswith(FULL):
                    st["valu4"] += 1
                    st["op:" + op] += 1
            elif op.startswith("ds_"):
                st["lds"] += 1
                if "permute" in op:
                    st["perm"] += 1
            elif op.startswith(("global_", "buffer_", "flat_")):
                st["vmem"] += 1
            elif op == "s_waitcnt":
                st["wait"] += 1
            elif op == "s_barrier":
                st["barrier"] += 1
            elif op.startswith(("s_cbranch", "s_branch")):
                st["branch"] += 1
            elif op.startswith("s_"):
                st["salu"] += 1
        for key in order + ["straight"]:
            st = stats[key]
            if not st:
                continue
            top = sorted(((v, k[3:]) for k, v in st.items() if k.startswith("op:")), reverse=True)[:12]
            print("%-16s valu %4d (4-cyc %4d) salu %4d lds %3d (perm %2d) vmem %3d wait %3d bar %d br %3d | %s" % (
                key, st["valu"], st["valu4"], st["salu"], st["lds"], st["perm"], st["vmem"], st["wait"],
                st["barrier"], st["branch"], " ".join("%s:%d" % (k, v) for v, k in top)))


if __name__ == "__main__":
    main()
