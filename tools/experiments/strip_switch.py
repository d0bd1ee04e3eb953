#!/usr/bin/env python3
"""Remove an experiment switch (an -D macro that is undefined in every measured build) from a source file, keeping
the code of the undefined case, and write the removed code as a patch that restores it.

    python tools/experiments/strip_switch.py FILE PATCH MACRO [MACRO ...]

Handled: `#ifdef M` / `#ifndef M` blocks (with an optional `#else`, nested directives inside are kept as text),
`defined(M) ||` terms of the product-build guard, and `#ifdef M` lines inside other #if blocks.  The patch is a unified
diff (stripped -> original) that `git apply` / `patch -p1` re-applies to the tree."""
from __future__ import annotations

import difflib
import os
import re
import sys


def strip(src: str, macros: set[str]) -> str:
    lines = src.split("\n")
    out = []
    # stack of (kind, keep_now, is_target): for target blocks keep_now tracks which branch is kept
    stack: list[list] = []

    def keeping() -> bool:
        return all(fr[1] for fr in stack if fr[2])

    for ln in lines:
        s = ln.strip()
        m = re.match(r"#\s*(ifdef|ifndef)\s+(\w+)", s)
        if m:
            tgt = m.group(2) in macros
            if tgt:
                # the switch is undefined: #ifdef → skip the first branch, #ifndef → keep it
                stack.append(["if", m.group(1) == "ifndef", True])
                continue
            stack.append(["if", True, False])
            if keeping():
                out.append(ln)
            continue
        if re.match(r"#\s*if\b", s):
            stack.append(["if", True, False])
            if keeping():
                out.append(ln)
            continue
        if re.match(r"#\s*(else|elif)\b", s):
            fr = stack[-1]
            if fr[2]:
                if s.startswith("#elif"):
                    raise SystemExit(f"#elif in a target block: {ln}")
                fr[1] = not fr[1]
                continue
            if keeping():
                out.append(ln)
            continue
        if re.match(r"#\s*endif\b", s):
            fr = stack.pop()
            if fr[2]:
                continue
            if keeping():
                out.append(ln)
            continue
        if keeping():
            out.append(ln)
    assert not stack, "unbalanced directives"
    return rebuild_guard("\n".join(out), macros)


def rebuild_guard(text: str, drop: set[str]) -> str:
    """The product-build guard (`#if !defined(FWAV_DEBUG_API) && (defined(A) || ... )` before its #error) without the
    dropped names, re-flowed to 120 columns."""
    head = "#if !defined(FWAV_DEBUG_API) && ("
    a = text.find(head)
    if a < 0:
        return text
    b = text.index("#error", a)
    names = [n for n in re.findall(r"defined\((\w+)\)", text[a + len(head):b]) if n not in drop]
    rows, cur = [], head
    for i, n in enumerate(names):
        term = f"defined({n})" + (" || " if i + 1 < len(names) else ")")
        if len(cur) + len(term) > 117:
            rows.append(cur.rstrip() + " \\")
            cur = "    "
        cur += term
    rows.append(cur)
    return text[:a] + "\n".join(rows) + "\n" + text[b:]


def main():
    path, patch, *macros = sys.argv[1:]
    src = open(path).read()
    new = strip(src, set(macros))
    rel = os.path.relpath(path, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    diff = difflib.unified_diff(new.splitlines(True), src.splitlines(True), f"a/{rel}", f"b/{rel}")
    with open(patch, "w") as f:
        f.writelines(diff)
    with open(path, "w") as f:
        f.write(new)
    print(f"{path}: {len(src.splitlines())} -> {len(new.splitlines())} lines; {patch} restores {', '.join(macros)}")


if __name__ == "__main__":
    main()
