#!/usr/bin/env python3
"""unifdef.py -- DESIGN TOOL: resolve preprocessor conditionals on known macros in place
(drops compiled-out experiment branches from a source file; conditionals on other macros
are kept as they are).

  python3 tools/unifdef.py FILE NAME=VALUE ... NAME=undef ...

`#ifndef X / #define X v / #endif` default blocks of a resolved macro are removed with the
macro; a resolved macro used outside conditionals is an error (the build shows it).
"""
import re
import sys


def main():
    path = sys.argv[1]
    known = {}
    for a in sys.argv[2:]:
        k, v = a.split("=", 1)
        known[k] = None if v == "undef" else v
    lines = open(path).read().split("\n")
    out = []
    # stack entries: (mode, taking, seen_true) ; mode 'keep' = unresolved conditional (emit
    # the directives), 'res' = resolved (drop the directives, emit the taken branch)
    stack = []

    def active():
        return all(e[1] for e in stack)

    def evaluate(expr):
        e = expr.split("//")[0].strip()
        e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: (
            "1" if known.get(m.group(1), "?") not in (None, "?") else
            "0" if m.group(1) in known else "UNKNOWN"), e)
        e = re.sub(r"defined\s+(\w+)", lambda m: (
            "1" if known.get(m.group(1), "?") not in (None, "?") else
            "0" if m.group(1) in known else "UNKNOWN"), e)

        def sub(m):
            w = m.group(0)
            if w in known:
                return known[w] if known[w] is not None else "0"
            return w
        e = re.sub(r"\b[A-Za-z_]\w*\b", sub, e)
        if re.search(r"[A-Za-z_]", e):
            return None
        e = e.replace("&&", " and ").replace("||", " or ")
        e = re.sub(r"!(?!=)", " not ", e)
        return bool(eval(e))

    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(r"#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)", s)
        if not m:
            if active():
                out.append(ln)
            i += 1
            continue
        d, rest = m.group(1), m.group(2)
        if d in ("if", "ifdef", "ifndef"):
            name = rest.split("//")[0].strip()
            if d == "ifdef":
                val = None if name not in known else known[name] is not None
            elif d == "ifndef":
                val = None if name not in known else known[name] is None
                # the default-value block of a resolved macro: drop it whole
                if name in known and i + 2 < len(lines) and \
                        re.match(r"#\s*define\s+%s\b" % re.escape(name), lines[i + 1].strip()) and \
                        re.match(r"#\s*endif", lines[i + 2].strip()):
                    i += 3
                    continue
            else:
                val = evaluate(rest)
            if val is None:
                stack.append(["keep", True, True])
                if active():
                    out.append(ln)
            else:
                stack.append(["res", val, val])
        elif d == "elif":
            top = stack[-1]
            if top[0] == "keep":
                if all(e[1] for e in stack[:-1]):
                    out.append(ln)
            else:
                val = evaluate(rest)
                if val is None:
                    raise SystemExit("line %d: #elif on unknown macros after a resolved #if" % (i + 1))
                top[1] = (not top[2]) and val
                top[2] = top[2] or val
        elif d == "else":
            top = stack[-1]
            if top[0] == "keep":
                if all(e[1] for e in stack[:-1]):
                    out.append(ln)
            else:
                top[1] = not top[2]
                top[2] = True
        else:  # endif
            top = stack.pop()
            if top[0] == "keep" and active():
                out.append(ln)
        i += 1
    assert not stack, "unbalanced conditionals"
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
