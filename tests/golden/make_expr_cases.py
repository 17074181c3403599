"""Regenerate tests/golden/expr_cases.json from the reference ExpressionTest known answers.

Reads src/common/filter/test/ExpressionTest.cpp as TEXT and keeps every
TEST_EXPR / _GT / _GE / _LT / _LE / _FAILED(expr, expected) whose expected value is a literal
(int / hex / double / bool / string, or the test's `minInt`). Cases that use nondeterministic
functions (rand32, rand64, now) or `expected` variables are skipped. The literal `expected`'s C++
type decides the compared variant type (Expression::as<decltype(expected)>), recorded as
int / double / bool / string.

    python tests/golden/make_expr_cases.py /root/reference
"""
import json
import os
import re
import sys

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
path = os.path.join(ref, "src/common/filter/test/ExpressionTest.cpp")
src = open(path).read()
lines = src.split("\n")


def split_args(s, i):
    """s[i] is just after '('. Return (args, end_index)."""
    depth, args, cur, q = 0, [], "", None
    while i < len(s):
        c = s[i]
        if q:
            cur += c
            if c == "\\":
                cur += s[i + 1]
                i += 2
                continue
            if c == q:
                q = None
        elif c in "\"'":
            q = c
            cur += c
        elif c == "(":
            depth += 1
            cur += c
        elif c == ")":
            if depth == 0:
                args.append(cur.strip())
                return args, i
            depth -= 1
            cur += c
        elif c == "," and depth == 0:
            args.append(cur.strip())
            cur = ""
        else:
            cur += c
        i += 1
    raise ValueError("unbalanced")


def literal(x):
    x = x.strip()
    if x in ("true", "false"):
        return "bool", x == "true"
    if x == "minInt":
        return "int", -(1 << 63)
    if re.fullmatch(r"-?0[xX][0-9a-fA-F]+", x):
        return "int", int(x, 16)
    if re.fullmatch(r"-?\d+", x):
        return "int", int(x)
    if re.fullmatch(r"-?(\d+\.\d*|\.\d+|\d+\.)([eE][-+]?\d+)?", x) or re.fullmatch(r"-?\d+[eE][-+]?\d+", x):
        return "double", float(x)
    m = re.fullmatch(r'(?:std::string\()?"((?:[^"\\]|\\.)*)"\)?', x)
    if m:
        return "string", m.group(1).encode().decode("unicode_escape")
    return None


cases, skipped = [], 0
for m in re.finditer(r"TEST_EXPR(_GT|_GE|_LT|_LE|_FAILED)?\(", src):
    line_no = src.count("\n", 0, m.start()) + 1
    if lines[line_no - 1].lstrip().startswith("#define"):
        continue
    args, _ = split_args(src, m.end())
    op = (m.group(1) or "_EQ")[1:]
    expr = args[0] if op == "FAILED" else ", ".join(args[:-1])
    expr = re.sub(r"\s+", " ", expr)
    if re.search(r"\b(rand32|rand64|now)\s*\(", expr):
        skipped += 1
        continue
    case = {"line": line_no, "op": op, "expr": expr}
    if op != "FAILED":
        lit = literal(args[-1])
        if lit is None:
            skipped += 1
            continue
        case["type"], case["expected"] = lit
    cases.append(case)

out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "expr_cases.json")
json.dump({"source": "src/common/filter/test/ExpressionTest.cpp", "cases": cases}, open(out, "w"), indent=0)
print(f"wrote {out}: {len(cases)} cases ({skipped} skipped)")
