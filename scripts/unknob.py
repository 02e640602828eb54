"""Resolve a source file's tuning knobs at their default values (a small
unifdef): every `#ifndef X / #define X v / #endif` default block of a macro
matching --knobs is removed, `#if/#ifdef/#ifndef/#elif` directives whose
condition only uses such knobs (or knobs that are never defined: diagnostic
switches) are evaluated and dropped with their dead branches, and remaining
uses of the knobs in code are replaced by their values.  Conditionals on any
other macro (JFS_PROF, ...) are kept.
usage: unknob.py <file> <regex of knob names> [--undef NAME...]"""
import re
import sys

path, pat = sys.argv[1], re.compile(sys.argv[2])
src = open(path).read().split("\n")

# 1. defaults
defaults = {}
i = 0
while i + 2 < len(src):
    a, b, c = src[i].strip(), src[i + 1].strip(), src[i + 2].strip()
    m1 = re.match(r"#ifndef\s+(\w+)$", a)
    m2 = re.match(r"#define\s+(\w+)\s+(.*?)\s*(//.*)?$", b)
    if m1 and m2 and m1.group(1) == m2.group(1) and c.startswith("#endif") and pat.fullmatch(m1.group(1)):
        defaults[m1.group(1)] = m2.group(2)
    i += 1


def known(name):
    return bool(pat.fullmatch(name))


def evaluate(expr):
    """True/False, or None when the expression uses a macro that is not a knob."""
    e = expr.split("//")[0].strip()
    names = set(re.findall(r"[A-Za-z_]\w*", e)) - {"defined"}
    if not names or not all(known(n) for n in names):
        return None
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if m.group(1) in defaults else "0", e)
    e = re.sub(r"defined\s+(\w+)", lambda m: "1" if m.group(1) in defaults else "0", e)
    e = re.sub(r"[A-Za-z_]\w*", lambda m: "(" + defaults.get(m.group(0), "0") + ")", e)
    e = e.replace("&&", " and ").replace("||", " or ").replace("!", " not ").replace(" not =", "!=")
    return bool(eval(e))


out = []
# stack entries: [kind, emitting_before, taken_any, current_taking] for resolved
# directives; ["keep"] for kept ones
stack = []


def emitting():
    return all(f[1] for f in stack if f[0] == "res") and all(f[3] for f in stack if f[0] == "res")


skip_default = 0
j = 0
while j < len(src):
    line = src[j]
    st = line.strip()
    # default blocks of knobs
    if j + 2 < len(src):
        m1 = re.match(r"#ifndef\s+(\w+)$", st)
        m2 = re.match(r"#define\s+(\w+)\s", src[j + 1].strip() + " ")
        if m1 and m2 and m1.group(1) == m2.group(1) and m1.group(1) in defaults and src[j + 2].strip().startswith("#endif"):
            j += 3
            continue
    m = re.match(r"#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$", st)
    if m:
        kw, rest = m.group(1), m.group(2).strip()
        if kw in ("if", "ifdef", "ifndef"):
            if kw == "if":
                v = evaluate(rest)
            else:
                name = rest.split()[0]
                v = None if not known(name) else ((name in defaults) == (kw == "ifdef"))
            if v is None:
                stack.append(["keep"])
                if emitting():
                    out.append(line)
            else:
                stack.append(["res", True, v, v])
            j += 1
            continue
        top = stack[-1]
        if kw == "elif":
            if top[0] == "keep":
                assert evaluate(rest) is None, f"mixed #elif at line {j + 1}"
                if emitting():
                    out.append(line)
            else:
                v = evaluate(rest)
                assert v is not None, f"unresolvable #elif at line {j + 1}"
                top[3] = (not top[2]) and v
                top[2] = top[2] or v
            j += 1
            continue
        if kw == "else":
            if top[0] == "keep":
                if emitting():
                    out.append(line)
            else:
                top[3] = not top[2]
                top[2] = True
            j += 1
            continue
        if kw == "endif":
            f = stack.pop()
            if f[0] == "keep" and emitting():
                out.append(line)
            j += 1
            continue
    if emitting():
        out.append(line)
    j += 1
assert not stack

text = "\n".join(out)
for k, v in sorted(defaults.items(), key=lambda kv: -len(kv[0])):
    text = re.sub(r"\b" + k + r"\b", v, text)
open(path, "w").write(text)
print(f"{len(defaults)} knobs resolved: " + ", ".join(f"{k}={v}" for k, v in sorted(defaults.items())))
