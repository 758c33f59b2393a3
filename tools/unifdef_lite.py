#!/usr/bin/env python3
"""Partial preprocessor for pruning build knobs out of the product sources (a small unifdef).

    tools/unifdef_lite.py FILE... -D NAME=VALUE ...

Every conditional whose expression only involves the given macros is resolved: the taken branch
is kept without its directives, the others are dropped (so `#ifndef QRK_X / #define QRK_X v /
#endif` knob definitions disappear).  Conditionals that still depend on other macros are kept,
with the given macros replaced by their values.  Ordinary code lines get the macros replaced by
their values too (runtime uses such as `if (QRK_X)` are then cleaned up by hand).  Files are
rewritten in place.
"""
import re
import sys

IDENT = re.compile(r"\b[A-Za-z_]\w*\b")


def subst(expr, known):
    expr = re.sub(r"defined\s*\(\s*(\w+)\s*\)|defined\s+(\w+)",
                  lambda m: ("1" if (m.group(1) or m.group(2)) in known else m.group(0)), expr)
    return IDENT.sub(lambda m: str(known[m.group(0)]) if m.group(0) in known else m.group(0), expr)


def evaluate(expr, known):
    """int value of a preprocessor expression over known macros, or None if it needs others"""
    e = re.sub(r"/\*.*?\*/", " ", expr.split("//")[0])
    e = subst(e, known).strip()
    if IDENT.search(e):
        return None
    py = e.replace("&&", " and ").replace("||", " or ")
    py = re.sub(r"!(?!=)", " not ", py)
    py = py.replace("/", "//")
    try:
        return int(eval(py, {}, {}))
    except Exception:
        return None


def process(lines, known):
    out = []
    # frame: [mode ('known'|'open'), taken, active, parent_active]
    stack = []

    def emitting():
        return all(f[2] and f[3] for f in stack) if stack else True

    for line in lines:
        m = re.match(r"\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$", line)
        if not m:
            if emitting():
                out.append(subst(line, known) if not line.lstrip().startswith("//") else line)
            continue
        d, rest = m.group(1), m.group(2).strip()
        parent = emitting()
        if d in ("if", "ifdef", "ifndef"):
            if d == "if":
                v = evaluate(rest, known)
            else:
                name = rest.split()[0]
                v = (name in known) if name in known else None
                if v is not None and d == "ifndef":
                    v = not v
            if v is None:
                stack.append(["open", False, True, parent])
                if parent:
                    out.append(line if d != "if" else line.replace(rest, subst(rest, known)))
            else:
                stack.append(["known", bool(v), bool(v), parent])
        elif d == "elif":
            f = stack[-1]
            if f[0] == "known":
                if f[1]:
                    f[2] = False
                else:
                    v = evaluate(rest, known)
                    if v is None:  # becomes an open conditional from here on
                        f[0], f[2] = "opened", True
                        if f[3]:
                            out.append(re.sub(r"#\s*elif", "#if", line).replace(rest, subst(rest, known)))
                    else:
                        f[2] = bool(v)
                        f[1] = bool(v)
            else:
                f[2] = True
                if f[3]:
                    out.append(line.replace(rest, subst(rest, known)))
        elif d == "else":
            f = stack[-1]
            if f[0] == "known":
                f[2] = not f[1]
                f[1] = True
            else:
                f[2] = True
                if f[3]:
                    out.append(line)
        else:  # endif
            f = stack.pop()
            if f[0] != "known" and f[3]:
                out.append(line)
    assert not stack, "unbalanced conditionals"
    return out


def main():
    args = sys.argv[1:]
    files, known = [], {}
    i = 0
    while i < len(args):
        if args[i] == "-D":
            k, v = args[i + 1].split("=", 1)
            known[k] = int(v)
            i += 2
        else:
            files.append(args[i])
            i += 1
    for fn in files:
        lines = open(fn).read().split("\n")
        open(fn, "w").write("\n".join(process(lines, known)))


if __name__ == "__main__":
    main()
