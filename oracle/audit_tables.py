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

Second check (check_case_conditions): the comparison above pairs the
reference's i-th `out = ...` statement with the oracle's case
(i // 16, i // 4 % 4, i % 4) = (z flag, tile case, position case).  That
pairing is only right if the oracle classifies a pixel into the case whose
reference branch conditions it satisfies.  So every reference branch path
(`z==0`, `tx==0&&ty==0`, `u==0`, `v>0`, ... and their negations) is evaluated
on every pixel of a 3 x 3-lens neighbourhood (T = 5) in both modes, and the
ONE path it satisfies must be the one the oracle's exported tile_case /
pos_case (lfmo_tile_case / lfmo_pos_case) select.  A permuted case order in
the oracle -- consistent across all 21 tables, which the first check would
miss -- fails here (tests/test_oracle.py mutation tests).

Usage: python oracle/audit_tables.py [/root/reference]
Exit status 0 when all 672 cases (3 families x 7 predictors x 2 modes x 16
cases) agree and every sampled pixel lands on its case.
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


def reference_paths(ref_root):
    """{(family, k): [32 branch paths]}: the full condition list (guard
    included) of each `out[...] = ...` statement, in source order."""
    paths = {}
    for fam, fname in FAMILIES:
        src = open(os.path.join(ref_root, "src", fname)).read()
        for k in range(1, 8):
            body = _strip_comments(_kernel_body(src, "_predictor%d_%s" % (k, fam)))
            items, _ = _parse_block(body, 0)
            rows = []
            _walk(items, [], rows)
            paths[(fam, k)] = [p for p, st in rows if st.startswith("out")]
    return paths


_COND_NAMES = {"z", "tx", "ty", "u", "v", "x", "y", "tileSize", "width", "height"}
_COND_NODES = (ast.Expression, ast.BoolOp, ast.And, ast.Or, ast.UnaryOp, ast.Not, ast.Compare, ast.Eq, ast.NotEq,
               ast.Lt, ast.LtE, ast.Gt, ast.GtE, ast.Name, ast.Load, ast.Constant)


def _condition(c):
    """A reference branch condition (C text) as a checked Python expression
    code object: only comparisons / and / or / not over the kernel's index
    variables and integer constants are accepted (the text is never executed
    in any other form)."""
    py = re.sub(r"!(?!=)", " not ", c.replace("&&", " and ").replace("||", " or "))
    tree = ast.parse(py.strip(), mode="eval")
    for node in ast.walk(tree):
        if not isinstance(node, _COND_NODES):
            raise ValueError("unexpected construct in reference condition %r" % c)
        if isinstance(node, ast.Name) and node.id not in _COND_NAMES:
            raise ValueError("unknown name %r in reference condition %r" % (node.id, c))
        if isinstance(node, ast.Constant) and not isinstance(node.value, int):
            raise ValueError("non-integer constant in reference condition %r" % c)
    return compile(tree, "<reference condition>", "eval")


def check_case_conditions(ref_root, tile_case, pos_case, T=5, paths=None):
    """(pixels checked, mismatches): for every kernel and every pixel of the
    lenses (tx, ty) in {0,1,2}^2, both modes, the index of the ONE reference
    branch path the pixel satisfies must equal
    z * 16 + tile_case(tx, ty) * 4 + pos_case(u, v)."""
    paths = paths or reference_paths(ref_root)
    compiled = {}
    bad = []
    n = 0
    for (fam, k), plist in sorted(paths.items()):
        code = [[compiled.setdefault(c, _condition(c)) for c in p] for p in plist]
        for z in (0, 1):
            for tx in range(3):
                for ty in range(3):
                    for u in range(T):
                        for v in range(T):
                            env = {"z": z, "tx": tx, "ty": ty, "u": u, "v": v, "x": u + tx * T, "y": v + ty * T,
                                   "tileSize": T, "width": 1 << 20, "height": 1 << 20}
                            hits = [i for i, p in enumerate(code)
                                    if all(eval(c, {"__builtins__": {}}, env) for c in p)]
                            exp = z * 16 + tile_case(tx, ty) * 4 + pos_case(u, v)
                            n += 1
                            if hits != [exp]:
                                bad.append((fam, k, z, tx, ty, u, v, hits, exp))
    return n, bad


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


def audit_conditions(ref_root, lib_path=None):
    lib = ctypes.CDLL(lib_path or os.path.join(HERE, "liblfm_oracle.so"))
    return check_case_conditions(ref_root, lib.lfmo_tile_case, lib.lfmo_pos_case)


def audit(ref_root, lib_path=None, texts=None):
    lib = ctypes.CDLL(lib_path or os.path.join(HERE, "liblfm_oracle.so"))
    texts = texts or oracle_formulas()
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
    nc, badc = audit_conditions(root)
    for b in badc[:20]:
        print("CASE MISMATCH fam=%s P%d z=%d tx=%d ty=%d u=%d v=%d: reference path(s) %s, oracle case %d" % b)
    print("checked %d pixels against the reference branch conditions, %d mismatches" % (nc, len(badc)))
    sys.exit(1 if bad or badc else 0)
