#!/usr/bin/env python3
"""Kill the YARN applications a Spark/Hadoop launch left behind (reference: bin/yarn_job_kill.py).

Scans a launcher log for ``application_<ts>_<id>`` ids and runs ``yarn application -kill``
on the last N distinct ones. This build trains with torch.distributed (one process per
GPU), so YARN is only involved when a site wraps the launchers in YARN itself; without a
``yarn`` binary the ids are printed and nothing is killed.
usage: bin/yarn_job_kill.py LOG_FILE [N=8]
"""
import re
import shutil
import subprocess
import sys


def main():
    if len(sys.argv) < 2:
        print(__doc__)
        return 2
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    ids = []
    for line in open(sys.argv[1], errors="replace"):
        for app in re.findall(r"application_\d+_\d+", line):
            if app not in ids:
                ids.append(app)
    ids = ids[-n:]
    yarn = shutil.which("yarn")
    for app in ids:
        if yarn:
            subprocess.run([yarn, "application", "-kill", app], check=False)
        else:
            print(f"yarn not found; would kill {app}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
