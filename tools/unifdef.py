"""Resolve chosen preprocessor conditionals of a source file (a small unifdef): every
#ifdef/#ifndef/#if on a macro in --defined / --undefined (or `#if NAME` with NAME given a value)
is replaced by the branch that macro selects; other directives are kept as they are.

  python tools/unifdef.py FILE -D VCRT_LEVELS_NF=1 -U VCRT_PAIR_FETCH > out

Used to strip measured-and-dropped experiments out of tracer.hip; the removed branches are kept
as patches under tools/experiments/ (git diff of the stripped file against the original)."""
import argparse
import re
import sys


def resolve(lines, defs, undefs):
    out, stack = [], []  # stack entries: (kind, keep_this_branch, resolved)

    def active():
        return all(k for _, k, _ in stack)

    for line in lines:
        s = line.strip()
        m = re.match(r"#\s*(ifdef|ifndef)\s+(\w+)", s)
        m2 = re.match(r"#\s*if\s+(!?)\s*(?:defined\s*\(?\s*)?(\w+)\s*\)?\s*$", s)
        if m or m2:
            if m:
                kind, name = m.group(1), m.group(2)
                neg = kind == "ifndef"
            else:
                name, neg = m2.group(2), bool(m2.group(1))
            if name in defs or name in undefs:
                if m or "defined" in s:
                    val = name in defs
                else:
                    val = name in defs and defs[name] not in ("0", "")
                stack.append(("r", val != neg, True))
                continue
            stack.append(("k", True, False))
            if active():
                out.append(line)
            continue
        if re.match(r"#\s*(if|ifdef|ifndef)\b", s):
            stack.append(("k", True, False))
            if active():
                out.append(line)
            continue
        if re.match(r"#\s*else\b", s):
            kind, keep, res = stack.pop()
            if res:
                stack.append((kind, not keep, True))
                continue
            stack.append((kind, keep, res))
            if active():
                out.append(line)
            continue
        if re.match(r"#\s*endif\b", s):
            kind, keep, res = stack.pop()
            if not res and active():
                out.append(line)
            continue
        if active():
            out.append(line)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("file")
    p.add_argument("-D", action="append", default=[])
    p.add_argument("-U", action="append", default=[])
    a = p.parse_args()
    defs = dict((d.split("=", 1) + ["1"])[:2] for d in a.D)
    sys.stdout.write("".join(resolve(open(a.file).readlines(), defs, set(a.U))))


if __name__ == "__main__":
    main()
