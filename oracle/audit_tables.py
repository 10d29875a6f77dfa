"""Text-level audit of the oracle's predictor case tables against the reference.

TEST INFRASTRUCTURE ONLY (see lfm_oracle.c header).

The reference kernels (lfm_Predictors.cu, lfm_Predictors_angle.cu,
lfm_Predictors_space.cu) cannot be compiled here (nvcc / cuda_runtime.h /
thrust are absent), so this script does not run them.  It reads their source
as text, walks the if/else tree of every `_predictorK_<family>` kernel, rewrites
each `out[p * y + x] = <expr>;` right-hand side into neighbour names
(I, A, B, C, Ap, Bp, Cp, Ap1, Bp1, ABp, BAp, P) and compares its parse tree with
the expression the oracle builds for the same case from its formula table and
temporal rule.  Python's `+ - >>` precedence equals C's, so equal parse trees
mean equal integer arithmetic.

Usage: python oracle/audit_tables.py [/root/reference]
Exit status 0 when all 672 cases (3 families x 7 predictors x 2 modes x 16
cases) agree.
"""
import ast
import ctypes
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
FAMILIES = [("tiles", "lfm_Predictors.cu"), ("angle", "lfm_Predictors_angle.cu"),
            ("space", "lfm_Predictors_space.cu")]

_NEIGHBOURS = {
    "p*y+x": "I", "p*y+x-1": "A", "p*(y-1)+x": "B", "p*(y-1)+x-1": "C",
    "p*y+x-tileSize": "Ap", "p*(y-tileSize)+x": "Bp", "p*(y-tileSize)+x-tileSize": "Cp",
    "width*height+p*y+x": "P", "p*y+x-tileSize-1": "Ap1", "p*(y-tileSize-1)+x": "Bp1",
    "p*(y-tileSize)+x-1": "ABp", "p*(y-1)+x-tileSize": "BAp",
}


def _strip_comments(s):
    s = re.sub(r"/\*.*?\*/", "", s, flags=re.S)
    return re.sub(r"//[^\n]*", "", s)


def _kernel_body(src, name):
    m = re.search(r"__global__\s+void\s+" + name + r"\s*\(", src)
    i = src.index("{", m.end())
    depth = 0
    for j in range(i, len(src)):
        if src[j] == "{":
            depth += 1
        elif src[j] == "}":
            depth -= 1
            if depth == 0:
                return src[i + 1:j]
    raise ValueError(name)


def _paren(s, pos):
    depth = 0
    for j in range(pos, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return s[pos + 1:j], j + 1
    raise ValueError("unbalanced")


def _parse_block(s, pos):
    items = []
    while True:
        while pos < len(s) and s[pos] in " \t\r\n;":
            pos += 1
        if pos >= len(s) or s[pos] == "}":
            return items, pos
        if re.match(r"if\s*\(", s[pos:]):
            branches, els = [], None
            while True:
                pos = s.index("(", pos)
                cond, pos = _paren(s, pos)
                pos = s.index("{", pos)
                blk, pos = _parse_block(s, pos + 1)
                pos += 1
                branches.append((re.sub(r"\s+", "", cond), blk))
                m = re.match(r"\s*else\s*", s[pos:])
                if not m:
                    break
                pos += m.end()
                if re.match(r"if\s*\(", s[pos:]):
                    continue
                pos = s.index("{", pos)
                els, pos = _parse_block(s, pos + 1)
                pos += 1
                break
            items.append(("if", branches, els))
        else:
            e = s.index(";", pos)
            items.append(("stmt", s[pos:e].strip()))
            pos = e + 1


def _walk(items, path, out):
    for it in items:
        if it[0] == "stmt":
            out.append((tuple(path), it[1]))
            continue
        _, branches, els = it
        neg = []
        for cond, blk in branches:
            _walk(blk, path + neg + [cond], out)
            neg = neg + ["!(" + cond + ")"]
        if els is not None:
            _walk(els, path + neg, out)


def _normalise(rhs):
    e = re.sub(r"\s+", "", rhs).replace("(int)", "")

    def rep(m):
        idx = m.group(1)
        if idx not in _NEIGHBOURS:
            raise ValueError("unknown neighbour index " + idx)
        return _NEIGHBOURS[idx]
    return re.sub(r"in\[([^\]]*)\]", rep, e)


# The case order every kernel uses (checked below): z==0 first, then the four
# tile cases, each with the four position cases.
_EXPECTED_PATHS = None


def reference_table(ref_root):
    """{(family, k): [32 normalised expressions]} in (z, tc, uc) order."""
    global _EXPECTED_PATHS
    table = {}
    for fam, fname in FAMILIES:
        src = open(os.path.join(ref_root, "src", fname)).read()
        for k in range(1, 8):
            body = _strip_comments(_kernel_body(src, "_predictor%d_%s" % (k, fam)))
            items, _ = _parse_block(body, 0)
            rows = []
            _walk(items, [], rows)
            paths = []
            exprs = []
            for path, st in rows:
                if not st.startswith("out"):
                    continue
                lhs, rhs = st.split("=", 1)
                assert re.sub(r"\s+", "", lhs) == "out[p*y+x]", lhs
                paths.append(tuple(c for c in path if not c.startswith("u>=0")))
                exprs.append(_normalise(rhs))
            assert len(exprs) == 32, (fam, k, len(exprs))
            if _EXPECTED_PATHS is None:
                _EXPECTED_PATHS = paths
            assert paths == _EXPECTED_PATHS, (fam, k, "case structure differs")
            table[(fam, k)] = exprs
    return table


def oracle_formulas():
    """formula id -> expression text, parsed from lfm_oracle.c."""
    src = open(os.path.join(HERE, "lfm_oracle.c")).read()
    enum_body = src[src.index("enum {"):src.index("F_NUM")]
    names = re.findall(r"\b(F_[A-Z0-9_]+)\b", re.sub(r"/\*.*?\*/", "", enum_body, flags=re.S))
    ids = {n: i for i, n in enumerate(names)}
    texts = {}
    for name, expr in re.findall(r"case (F_[A-Z0-9_]+): return (.*?);", src):
        texts[ids[name]] = expr
    return texts


def oracle_expression(lib, texts, fam_idx, k, zflag, tc, uc):
    f = lib.lfmo_case_formula(fam_idx, k, tc, uc)
    pred = texts[f]
    if not zflag:
        return "I" if pred == "0" else "I-(%s)" % pred
    if pred == "0":
        return "I-P"
    if fam_idx == 0:
        return "I-(((%s)+P)>>1)" % pred
    if lib.lfmo_case_temporal_double(fam_idx, k, tc, uc):
        return "((((I-(%s))+P)>>1)+P)>>1" % pred
    return "((I-(%s))+P)>>1" % pred


def audit(ref_root, lib_path=None):
    lib = ctypes.CDLL(lib_path or os.path.join(HERE, "liblfm_oracle.so"))
    texts = oracle_formulas()
    ref = reference_table(ref_root)
    bad = []
    n = 0
    for fi, (fam, _) in enumerate(FAMILIES):
        for k in range(1, 8):
            for zflag in (0, 1):
                for tc in range(4):
                    for uc in range(4):
                        r = ref[(fam, k)][zflag * 16 + tc * 4 + uc]
                        o = oracle_expression(lib, texts, fi, k, zflag, tc, uc)
                        n += 1
                        if ast.dump(ast.parse(r, mode="eval")) != ast.dump(ast.parse(o, mode="eval")):
                            bad.append((fam, k, zflag, tc, uc, r, o))
    return n, bad


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    n, bad = audit(root)
    for b in bad:
        print("MISMATCH fam=%s P%d z=%d tc=%d uc=%d\n  ref:    %s\n  oracle: %s" % b)
    print("audited %d cases, %d mismatches" % (n, len(bad)))
    sys.exit(1 if bad else 0)
