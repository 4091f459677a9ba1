"""Minimal unifdef for the kernel sources: resolve #ifdef / #ifndef / #if
blocks whose condition is a single known macro (optionally negated, or
compared with == / != to an integer), keep everything else verbatim.

    python tools/unifdef.py FILE -DNAME=VALUE -UNAME ...

-D NAME=V: NAME is defined with integer value V; -U NAME: NAME is undefined.
A `#ifndef NAME / #define NAME V / #endif` default block of a -D macro is
dropped (its value becomes a literal in the resolved #if lines only; C++
uses of NAME must be replaced by hand).  Rewrites FILE in place."""
import re
import sys


def parse_args(argv):
    path, known = argv[0], {}
    for a in argv[1:]:
        if a.startswith("-D"):
            k, _, v = a[2:].partition("=")
            known[k] = int(v or "1")
        elif a.startswith("-U"):
            known[a[2:]] = None
    return path, known


def cond_value(line, known):
    """True / False if the directive's condition is decidable, else None."""
    m = re.match(r"\s*#\s*ifdef\s+(\w+)\s*$", line)
    if m:
        k = m.group(1)
        return None if k not in known else known[k] is not None
    m = re.match(r"\s*#\s*ifndef\s+(\w+)\s*$", line)
    if m:
        k = m.group(1)
        return None if k not in known else known[k] is None
    m = re.match(r"\s*#\s*if\s+(!?)\s*(\w+)\s*(?:(==|!=)\s*(\d+))?\s*$", line)
    if m:
        neg, k, op, v = m.groups()
        if k not in known:
            return None
        val = known[k] or 0
        r = (val == int(v)) if op == "==" else (val != int(v)) if op == "!=" else bool(val)
        return not r if neg else r
    m = re.match(r"\s*#\s*if\s+defined\s*\(?\s*(\w+)\s*\)?\s*$", line)
    if m:
        k = m.group(1)
        return None if k not in known else known[k] is not None
    return None


def main():
    path, known = parse_args(sys.argv[1:])
    lines = open(path).read().split("\n")
    out = []
    # stack entries: (decided, keep_current_branch, parent_emitting)
    stack = []

    def emitting():
        return all(e[1] if e[0] else True for e in stack) if stack else True

    for ln in lines:
        s = ln.strip()
        if re.match(r"#\s*if", s):
            cv = cond_value(ln, known)
            par = emitting()
            if cv is None:
                stack.append((False, True, par))
                if par:
                    out.append(ln)
            else:
                stack.append((True, cv, par))
            continue
        if re.match(r"#\s*elif", s):
            top = stack[-1]
            if top[0]:
                raise SystemExit("%s: #elif inside a resolved block is not supported" % path)
            if emitting():
                out.append(ln)
            continue
        if re.match(r"#\s*else", s):
            top = stack[-1]
            if top[0]:
                stack[-1] = (True, not top[1], top[2])
            elif emitting():
                out.append(ln)
            continue
        if re.match(r"#\s*endif", s):
            top = stack.pop()
            if not top[0] and emitting():
                out.append(ln)
            continue
        if emitting():
            out.append(ln)
    assert not stack, "unbalanced #if in %s" % path
    # drop the now-empty default blocks "#define NAME V" of -D macros
    text = "\n".join(out)
    for k, v in known.items():
        if v is not None:
            text = re.sub(r"\n#\s*define\s+%s\s+[^\n]*" % re.escape(k), "", text)
    open(path, "w").write(text)


if __name__ == "__main__":
    main()
