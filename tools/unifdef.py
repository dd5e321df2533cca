"""Resolve preprocessor conditionals on a fixed set of macros (a small `unifdef -D`).

    python tools/unifdef.py -DNWC_X=1 -DNWC_Y=0 file...     # rewrites the files in place

Conditionals whose expression names only the given macros are evaluated and removed, keeping the
taken branch; `#ifndef M` / `#ifdef M` of a given macro are resolved as "defined"; everything
else is kept verbatim.  Used to drop measured-and-rejected build switches from the product
sources (the measurements stay in profiles/*/experiments.md and git history).
"""
import re
import sys

ID = re.compile(r"[A-Za-z_]\w*")


def evaluate(expr, macros):
    names = set(ID.findall(expr)) - {"defined"}
    if not names or not names <= set(macros):
        return None
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if m.group(1) in macros else "0", expr)
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    e = ID.sub(lambda m: str(macros[m.group(0)]) if m.group(0) in macros else m.group(0), e)
    return bool(eval(e, {}, {}))


def process(lines, macros):
    out = []
    # stack entries: [mode, taken_already, keep_current]
    #   mode "keep": directive kept verbatim; "resolved": directives dropped, branch chosen
    stack = []

    def emitting():
        return all(s[2] for s in stack)

    for line in lines:
        m = re.match(r"\s*#\s*(ifndef|ifdef|if|elif|else|endif)\b(.*)", line)
        if not m:
            if emitting():
                out.append(line)
            continue
        d, rest = m.group(1), m.group(2).split("//")[0].strip()
        if d in ("if", "ifdef", "ifndef"):
            if d == "ifdef":
                v = True if rest in macros else None
            elif d == "ifndef":
                v = False if rest in macros else None
            else:
                v = evaluate(rest, macros)
            if v is None:
                stack.append(["keep", False, True])
                if emitting():
                    out.append(line)
            else:
                stack.append(["resolved", v, v])
        elif d == "elif":
            top = stack[-1]
            if top[0] == "keep":
                if all(s[2] for s in stack[:-1]):
                    out.append(line)
                continue
            if top[1]:
                top[2] = False
            else:
                v = evaluate(rest, macros)
                if v is None:
                    raise SystemExit("unresolvable #elif after resolved #if: " + line)
                top[1], top[2] = v, v
        elif d == "else":
            top = stack[-1]
            if top[0] == "keep":
                if all(s[2] for s in stack[:-1]):
                    out.append(line)
                continue
            top[2] = not top[1]
            top[1] = True
        else:  # endif
            top = stack.pop()
            if top[0] == "keep" and emitting():
                out.append(line)
    assert not stack, "unbalanced conditionals"
    return out


def main():
    macros, files = {}, []
    for a in sys.argv[1:]:
        if a.startswith("-D"):
            k, _, v = a[2:].partition("=")
            macros[k] = int(v or "1")
        else:
            files.append(a)
    for f in files:
        lines = open(f).read().split("\n")
        new = process(lines, macros)
        open(f, "w").write("\n".join(new))


if __name__ == "__main__":
    main()
