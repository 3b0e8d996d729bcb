"""Copy one report block of the reference's own output file (rezultat.txt,
lines 80-104: the 50-clause / 10-variable comparison) into
tests/golden/rezultat_block.txt -- a data fixture for the report-format test.

    python tests/golden/make_report_fixture.py
"""
import os

SRC = "/root/reference/rezultat.txt"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rezultat_block.txt")

if __name__ == "__main__":
    lines = open(SRC, encoding="utf-8").read().split("\n")
    with open(OUT, "w") as fh:
        fh.write("\n".join(lines[79:104]) + "\n")
