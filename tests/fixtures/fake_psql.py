#!/usr/bin/env python3
"""Stand-in for `psql -f -` in the native DbSink tests: reads `COPY t (cols) FROM STDIN;` blocks
terminated by `\\.`, appends the rows to $FAKE_PSQL_OUT/<table>.rows, and answers
`\\echo APMACK <n> :ERROR` with `APMACK <n> false` (or `true` for the table named in
$FAKE_PSQL_FAIL, whose rows are then not kept)."""
import os
import sys

out_dir = os.environ["FAKE_PSQL_OUT"]
fail = os.environ.get("FAKE_PSQL_FAIL", "")
hang = os.environ.get("FAKE_PSQL_HANG", "")  # commits this table's rows, then never acknowledges
table, rows, err, last = None, [], False, None
for line in sys.stdin:
    if table is not None:
        if line == "\\.\n":
            err = table == fail
            last = table
            if not err:
                with open(os.path.join(out_dir, table + ".rows"), "a") as f:
                    f.write("".join(rows))
            table, rows = None, []
        else:
            rows.append(line)
        continue
    if line.startswith("COPY "):
        if not globals().get("_seen"):
            _seen = True  # one line per connection: the writer-lane tests count them
            with open(os.path.join(out_dir, "connections"), "a") as f:
                f.write(f"{os.getpid()}\n")
        table = line.split()[1]
    elif line.startswith("\\echo APMACK"):
        if hang and last == hang:
            import time
            time.sleep(60)
        n = line.split()[2]
        sys.stdout.write(f"APMACK {n} {'true' if err else 'false'}\n")
        sys.stdout.flush()
