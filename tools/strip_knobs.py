"""Selective unifdef: resolve #if/#ifdef/#ifndef/#elif/#else/#endif whose conditions use only the
given macros (with the given values; None = undefined), keep every other directive untouched.

    python tools/strip_knobs.py FILE W4_STAGE_EPI=0 W4_DESYNC= ...   (in place)
"""
import re
import sys


def evaluate(cond, known):
    names = set(re.findall(r"\b[A-Za-z_]\w*\b", cond)) - {"defined"}
    if not names or not names <= set(known):
        return None
    expr = re.sub(r"defined\s*\(\s*(\w+)\s*\)|defined\s+(\w+)",
                  lambda m: "1" if known[m.group(1) or m.group(2)] is not None else "0", cond)
    expr = re.sub(r"\b([A-Za-z_]\w*)\b", lambda m: str(known[m.group(1)] or 0), expr)
    expr = expr.replace("&&", " and ").replace("||", " or ")
    expr = re.sub(r"!(?!=)", " not ", expr)
    return bool(eval(expr))


def strip(lines, known):
    out = []
    # stack entries: [resolved?, taking-now?, any-branch-taken?, parent-active?]
    stack = []
    active = lambda: all(e[1] for e in stack if e[0]) and all(e[3] for e in stack)  # noqa: E731
    for ln in lines:
        m = re.match(r"\s*#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)", ln)
        if not m:
            if active():
                out.append(ln)
            continue
        kw, rest = m.group(1), re.sub(r"//.*|/\*.*?\*/", "", m.group(2)).strip()
        if kw in ("if", "ifdef", "ifndef"):
            parent = active()
            if kw == "ifdef":
                v = (rest in known) and (known[rest] is not None) if rest in known else None
            elif kw == "ifndef":
                v = (known[rest] is None) if rest in known else None
            else:
                v = evaluate(rest, known)
            if v is None:
                stack.append([False, True, False, parent])
                if parent:
                    out.append(ln)
            else:
                stack.append([True, v, v, parent])
        elif kw == "elif":
            top = stack[-1]
            if not top[0]:
                if top[3]:
                    out.append(ln)
                continue
            v = evaluate(rest, known)
            if v is None:
                raise SystemExit(f"unresolvable #elif after a resolved #if: {ln!r}")
            top[1] = v and not top[2]
            top[2] = top[2] or v
        elif kw == "else":
            top = stack[-1]
            if not top[0]:
                if top[3]:
                    out.append(ln)
                continue
            top[1] = not top[2]
            top[2] = True
        else:
            top = stack.pop()
            if not top[0] and top[3]:
                out.append(ln)
    assert not stack
    return out


if __name__ == "__main__":
    path = sys.argv[1]
    known = {}
    for a in sys.argv[2:]:
        k, v = a.split("=", 1)
        known[k] = int(v) if v else None
    with open(path) as fh:
        lines = fh.readlines()
    with open(path, "w") as fh:
        fh.writelines(strip(lines, known))
