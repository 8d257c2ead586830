"""Exit cost of a process by what it holds (tools/ubench/exit_cost.cpp):
seconds from its last line to the parent seeing it exit."""
import os
import subprocess
import sys
import time

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "exit_cost")
for dev_gb, host_gb, mode in [(0, 0, 0), (150, 0, 0), (40, 0, 0), (0, 3, 0), (0, 3, 1), (150, 3, 1)]:
    for rep in range(2):
        time.sleep(4)  # the driver clears what the previous run freed
        p = subprocess.run([EXE, str(dev_gb), str(host_gb), str(mode)], stdout=subprocess.PIPE, text=True)
        t1 = time.time()
        if p.returncode != 0:
            print(f"dev {dev_gb} GB host {host_gb} GB mode {mode}: rc {p.returncode}", flush=True)
            continue
        print(f"dev {dev_gb} GB host {host_gb} GB mode {mode}: exit {t1 - float(p.stdout.split()[-1]):.3f} s", flush=True)
