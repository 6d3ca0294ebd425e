#!/usr/bin/env python3
"""Dump the table / view schema of a rocprofv3 rocpd database and two sample rows of
each, so the counter tools can join counters to the SAME pass's dispatch durations.
usage: rocpd_schema.py DB"""
import sqlite3
import sys

cur = sqlite3.connect(sys.argv[1]).cursor()
for name, kind in cur.execute("select name, type from sqlite_master where type in ('table','view') "
                              "order by type, name").fetchall():
    cols = [r[1] for r in cur.execute(f"pragma table_info('{name}')").fetchall()]
    print(f"{kind} {name}: {cols}")
    if any(s in name for s in ("kernel", "counter", "pmc", "dispatch")):
        try:
            for row in cur.execute(f"select * from '{name}' limit 2").fetchall():
                print("   ", str(row)[:400])
        except sqlite3.Error as e:
            print("    error", e)
