#!/usr/bin/env python3
"""The C-ABI entry-point table of INTEGRATION.md §4, generated from include/laspj.h (and the
A/B knob header include/laspj_tune.h):
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
HDRS = [os.path.join(ROOT, "include", h) for h in ("laspj.h", "laspj_tune.h")]
DOC = os.path.join(ROOT, "INTEGRATION.md")
BEGIN = "<!-- abi-table:begin (tools/abi_table.py --write) -->"
END = "<!-- abi-table:end -->"

DECL = re.compile(r"^\s*(?:const\s+)?[a-zA-Z_][\w\s\*]*?\b(laspj_\w+)\s*\(")
CITE = re.compile(r"\b[\w/]+\.(?:erl|hrl):\d+(?:-\d+)?(?:,\s*\d+(?:-\d+)?)*")


def entries():
    """(name, where, section, citations, first sentence) per declared function.  A comment
    block documents the declarations after it up to the next blank line or comment."""
    out = []
    for hdr in HDRS:
        out += _entries(hdr)
    return out


def _entries(hdr):
    lines = open(hdr).read().splitlines()
    base = os.path.basename(hdr)
    out, comment = [], []
    section = "" if base == "laspj.h" else "A/B knobs"
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
            out.append((m.group(1), no if base == "laspj.h" else f"{base}:{no}", section,
                        cites, first))
    return out


PLUMBING = ("library / context", "device buffers", "timing", "A/B knobs")


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
