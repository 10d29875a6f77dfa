"""Count instructions per kernel of an assembly file (hipcc -S), optionally
only between the `; ROW_BEGIN` / `; ROW_END` markers (scripts/isa_rows.hip).

python scripts/isa_count.py file.s [--rows]"""
import re
import subprocess
import sys


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and line.startswith(".Lfunc_end"):
            yield cur, body
            cur = None
            continue
        if cur:
            body.append(line)


def demangle(n):
    try:
        return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


def main():
    path = sys.argv[1]
    rows = "--rows" in sys.argv
    for name, body in kernels(path):
        if rows:
            inside, sel = False, []
            for ln in body:
                if "ROW_BEGIN" in ln:
                    inside = True
                elif "ROW_END" in ln:
                    inside = False
                elif inside:
                    sel.append(ln)
            body = sel
        ins = [ln.split()[0] for ln in body if re.match(r"^\s+[vsdgb][a-z_0-9]+", ln)]
        valu = [i for i in ins if i.startswith("v_")]
        pk = [i for i in valu if i.startswith("v_pk_")]
        salu = [i for i in ins if i.startswith("s_")]
        print("%-70s valu %4d (pk %3d) salu %3d total %4d" % (demangle(name)[:70], len(valu), len(pk), len(salu),
                                                                len(ins)))


if __name__ == "__main__":
    main()
