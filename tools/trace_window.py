#!/usr/bin/env python3
"""Print the last N kernel / copy events of a rocprofv3 SQLite trace with start times
relative to the first of them (microseconds) — to read one call's device timeline."""
import sqlite3
import sys


def short(name):
    n = str(name).replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].replace("laspj::", "")[:48]


def main(db, last):
    c = sqlite3.connect(db)
    ev = [(s, e, short(n)) for s, e, n in c.execute("select start, end, name from kernels")]
    try:
        ev += [(s, e, "COPY %s %d" % (str(n).replace("MEMORY_COPY_", ""), sz))
               for s, e, n, sz in c.execute("select start, end, name, size from memory_copies")]
    except sqlite3.OperationalError:
        pass
    ev.sort()
    ev = ev[-last:]
    t0 = ev[0][0]
    for s, e, n in ev:
        print("%9.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, n))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
