#!/usr/bin/env python3
"""The C-ABI entry-point table of INTEGRATION.md §4, generated from include/laspj.h:
every function the header declares, where (laspj.h:line), the reference function(s) its
comment block cites (file.erl:lines), and the comment's first sentence.  Functions whose
comment cites nothing are runtime plumbing (contexts, buffers, events, tuning).

    python tools/abi_table.py            # print the table
    python tools/abi_table.py --write    # replace §4 of INTEGRATION.md with it
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "laspj.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")
BEGIN = "<!-- abi-table:begin (tools/abi_table.py --write) -->"
END = "<!-- abi-table:end -->"

DECL = re.compile(r"^\s*(?:const\s+)?[a-zA-Z_][\w\s\*]*?\b(laspj_\w+)\s*\(")
CITE = re.compile(r"\b[\w/]+\.(?:erl|hrl):\d+(?:-\d+)?(?:,\s*\d+(?:-\d+)?)*")


def entries():
    """(name, line, section, citations, first sentence) per declared function.  A comment
    block documents the declarations after it up to the next blank line or comment."""
    lines = open(HDR).read().splitlines()
    out, comment, section = [], [], ""
    in_c = prev_comment = False
    for no, line in enumerate(lines, 1):
        s = line.strip()
        m = re.match(r"/\* -+ (.+?) \*/", s)
        if m:
            section, comment, prev_comment = m.group(1).strip(), [], False
            continue
        if s.startswith("/*") or in_c:
            if not in_c and not prev_comment:
                comment = []
            in_c = not s.endswith("*/")
            comment.append(s.strip("/* ").strip())
            prev_comment = True
            continue
        prev_comment = False
        if not s or s.startswith("#"):
            comment = []
            continue
        m = DECL.match(line)
        if m and not s.startswith("typedef"):
            text = " ".join(c for c in comment if c)
            cites = sorted(set(CITE.findall(text)), key=text.index)
            first = re.split(r"(?<=[.;])\s", text, maxsplit=1)[0] if text else ""
            out.append((m.group(1), no, section, cites, first))
    return out


PLUMBING = ("library / context", "device buffers", "timing")


def table():
    rows = ["| entry point | laspj.h | section | reference it serves | what |",
            "|---|---|---|---|---|"]
    for name, no, section, cites, first in entries():
        ref = "; ".join(cites) if cites else \
            ("(runtime plumbing)" if section in PLUMBING else "—")
        first = first.replace("|", "\\|")
        if len(first) > 110:
            first = first[:107].rstrip() + "..."
        rows.append(f"| `{name}` | {no} | {section} | {ref} | {first} |")
    return "\n".join(rows)


def main():
    t = table()
    if "--write" not in sys.argv:
        print(t)
        return
    doc = open(DOC).read()
    i, j = doc.index(BEGIN) + len(BEGIN), doc.index(END)
    open(DOC, "w").write(doc[:i] + "\n" + t + "\n" + doc[j:])


if __name__ == "__main__":
    main()
