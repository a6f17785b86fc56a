#!/usr/bin/env python3
"""Remove compile-time experiment switches from the product sources (a small
unifdef): every macro in UNDEF is taken as not defined, and each #if / #ifdef
/ #ifndef / #elif whose condition is decided by that is resolved -- the
losing branch and the directive lines go, other conditions keep their
directives with the decided terms simplified away.

    python tools/strip_switches.py FILE [FILE ...]      (rewrites in place)

Used once in round 4; the removed variants are kept as
tools/experiments/round3_switches.patch (`git apply` restores them)."""
import re
import sys

UNDEF = {
    "STL_NO_FE_FENCE", "STL_NO_ACC_FENCE", "STL_EXP_TABLE_ENTRIES", "STL_SHA_ADD64", "STL_SHA_FENCE",
    "STL_NO_LAZY_DBL", "STL_POINT_PAIRED", "STL_EXP_ENTRY0", "STL_NO_TABLE_PREFETCH", "STL_ID_CONST",
    "STL_EXP_HALF_FOOTPRINT", "STL_NT_STATE", "STL_PAIR_SHFL", "STL_WIDE_PACKED", "STL_TAILS_GLOBAL",
    "STL_WIDE_GLOBAL", "STL_WHOLE_PAIRED", "STL_POINT_PAIR_ALL", "STL_NO_JOINT", "STL_MAIN_NUM_VGPR",
}
VALUES = {"STL_GE_NOPS": 4}


def simplify(cond):
    """-> True / False when decided, else the condition with decided
    defined() terms replaced (still a string)."""
    c = cond
    for m in UNDEF:
        c = re.sub(r"!\s*defined\s*\(\s*%s\s*\)" % m, "1", c)
        c = re.sub(r"defined\s*\(\s*%s\s*\)" % m, "0", c)
        c = re.sub(r"!\s*defined\s+%s\b" % m, "1", c)
        c = re.sub(r"defined\s+%s\b" % m, "0", c)
    for m, v in VALUES.items():
        c = re.sub(r"\b%s\b" % m, str(v), c)
    try:
        py = c.replace("&&", " and ").replace("||", " or ")
        py = re.sub(r"!(?!=)", " not ", py)
        return bool(eval(py, {"__builtins__": {}}, {}))
    except Exception:  # noqa: BLE001 - undecided: other macros remain
        pass
    # drop decided operands of a flat && chain
    parts = [p.strip() for p in c.split("&&")]
    if len(parts) > 1 and "||" not in c:
        if any(p == "0" for p in parts):
            return False
        keep = [p for p in parts if p != "1"]
        return " && ".join(keep) if keep else True
    return c


def process(lines):
    out = []
    stack = []  # frames: [emit_parent, branch_taken, keep_directives, current_emit]

    def emitting():
        return all(f[3] for f in stack)

    for ln in lines:
        s = ln.strip()
        m = re.match(r"#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)", s)
        if not m:
            if emitting():
                out.append(ln)
            continue
        kw, rest = m.group(1), m.group(2).strip()
        rest = re.sub(r"//.*$", "", rest).strip()
        if kw in ("ifdef", "ifndef", "if"):
            if kw == "ifdef":
                cond = f"defined({rest})"
            elif kw == "ifndef":
                cond = f"!defined({rest})"
            else:
                cond = rest
            v = simplify(cond)
            if v is True or v is False:
                stack.append([emitting(), v, False, v])
            else:
                stack.append([emitting(), None, True, True])
                if emitting():
                    out.append(ln if kw != "if" or v == cond else ln.replace(rest, v))
            continue
        f = stack[-1]
        if kw == "elif":
            if not f[2]:
                if f[1]:
                    f[3] = False
                else:
                    v = simplify(rest)
                    if v is True or v is False:
                        f[1], f[3] = v, v
                    else:  # an undecided #elif after decided-false branches becomes an #if
                        f[2], f[1], f[3] = True, None, True
                        if f[0]:
                            out.append(ln.replace("#elif", "#if", 1).replace(rest, v))
            else:
                if f[0]:
                    out.append(ln)
            continue
        if kw == "else":
            if not f[2]:
                f[3] = not f[1]
            elif f[0]:
                out.append(ln)
            continue
        if kw == "endif":
            stack.pop()
            if f[2] and f[0]:
                out.append(ln)
    assert not stack, "unbalanced conditionals"
    return out


def main(paths):
    for p in paths:
        with open(p) as fh:
            lines = fh.readlines()
        new = process(lines)
        if new != lines:
            with open(p, "w") as fh:
                fh.writelines(new)
            print(f"{p}: {len(lines)} -> {len(new)} lines")


if __name__ == "__main__":
    main(sys.argv[1:])
