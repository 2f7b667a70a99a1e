"""Partial preprocessor for retiring build knobs: every macro named on the
command line is fixed at the value its `#ifndef X / #define X v / #endif`
default gives (or NAME=VALUE), its conditionals are resolved, its default
block is dropped and remaining uses are replaced by the value.  Conditionals
on other macros are kept as they are.
  python tools/unifdef.py FILE MACRO[=VALUE] ...   (rewrites FILE)"""
import re
import sys


def main():
    path = sys.argv[1]
    fixed = {}
    for a in sys.argv[2:]:
        k, _, v = a.partition("=")
        fixed[k] = v or None
    lines = open(path).read().split("\n")
    # 1. defaults: #ifndef X / #define X v [// comment] / #endif
    out, i = [], 0
    while i < len(lines):
        m = re.match(r"#ifndef (\w+)\s*$", lines[i])
        if m and m.group(1) in fixed and i + 2 < len(lines):
            d = re.match(r"#define (\w+)\s+(.*?)\s*(//.*)?$", lines[i + 1])
            j = i + 1
            # (a define continued by further comment lines)
            while j + 1 < len(lines) and lines[j + 1].lstrip().startswith("//"):
                j += 1
            if d and d.group(1) == m.group(1) and lines[j + 1].strip() == "#endif":
                if fixed[m.group(1)] is None:
                    fixed[m.group(1)] = d.group(2)
                i = j + 2
                continue
        out.append(lines[i])
        i += 1
    for k, v in fixed.items():
        assert v is not None, f"{k}: no default found and no value given"
    lines = out

    def subst(expr):
        for k, v in fixed.items():
            expr = re.sub(r"\b%s\b" % k, "(%s)" % v, expr)
        return expr

    def evaluable(expr):
        e = re.sub(r"defined\s*\(?\s*(\w+)\s*\)?", lambda m: "1" if m.group(1) in fixed else "UNKNOWN", expr)
        e = subst(e)
        if re.search(r"[A-Za-z_]", e.replace("and", "").replace("or", "").replace("not", "")):
            return None
        e = e.replace("&&", " and ").replace("||", " or ").replace("!", " not ").replace(" not =", "!=")
        try:
            return bool(eval(e))
        except Exception:
            return None

    # 2. conditionals: stack of (kind, keep-state); kind 'fixed' or 'other'
    res, stack = [], []

    def live():
        return all(s[1] for s in stack if s[0] == "fixed")

    for ln in lines:
        s = ln.strip()
        m = re.match(r"#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)", s)
        if m:
            kw, rest = m.group(1), m.group(2).strip()
            if kw in ("if", "ifdef", "ifndef"):
                expr = rest if kw == "if" else (f"defined({rest})" if kw == "ifdef" else f"!defined({rest})")
                v = evaluable(expr)
                if v is None:
                    stack.append(["other", True, False])
                    if live():
                        res.append(ln)
                else:
                    stack.append(["fixed", v, v])
                continue
            if kw == "elif":
                top = stack[-1]
                if top[0] == "other":
                    if live():
                        res.append(ln)
                    continue
                v = evaluable(rest)
                assert v is not None, ln
                top[1] = (not top[2]) and v
                top[2] = top[2] or v
                continue
            if kw == "else":
                top = stack[-1]
                if top[0] == "other":
                    if live():
                        res.append(ln)
                    continue
                top[1] = not top[2]
                top[2] = True
                continue
            if kw == "endif":
                top = stack.pop()
                if top[0] == "other" and live():
                    res.append(ln)
                continue
        if live():
            res.append(ln)
    assert not stack
    text = "\n".join(res)
    for k, v in fixed.items():
        text = re.sub(r"\b%s\b" % k, v, text)
    open(path, "w").write(text)


if __name__ == "__main__":
    main()
