#!/usr/bin/env python3
"""Run a command, print its wall time as one JSON line to stderr, exit with
its status (a measurement helper: the driver's own clock around a bench run).
  usage: python3 tools/wall.py OUT.json CMD [ARGS...]   (CMD's stdout passes through)"""
import json
import subprocess
import sys
import time

t0 = time.perf_counter()
rc = subprocess.call(sys.argv[2:])
json.dump({"cmd": " ".join(sys.argv[2:]), "rc": rc, "wall_s": round(time.perf_counter() - t0, 2)},
          open(sys.argv[1], "w"))
sys.exit(rc)
