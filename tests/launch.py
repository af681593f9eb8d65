"""torchrun launcher of the multi-process GPU tests: a fresh loopback port per
attempt, and one retry with another port when the rendezvous server could not
bind its port (EADDRINUSE: the port picked by bind(0) was taken again before
torchrun listened on it -- a launcher race, not a result of the test)."""
import os
import socket
import subprocess
import sys


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def torchrun(nproc, args, cwd, timeout, log_path, env=None, attempts=2):
    """Run `python -m torch.distributed.run ... args`; stdout+stderr go to
    log_path (and are echoed); returns the CompletedProcess of the last try."""
    r = None
    for _ in range(attempts):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr=127.0.0.1", f"--master-port={free_port()}"] + list(args)
        with open(log_path, "w") as f:
            r = subprocess.run(cmd, cwd=cwd, stdout=f, stderr=subprocess.STDOUT, timeout=timeout,
                               env=env if env is not None else os.environ.copy())
        text = open(log_path, errors="replace").read()
        print(text[-4000:], flush=True)
        if r.returncode == 0 or "EADDRINUSE" not in text:
            break
    r.log = open(log_path, errors="replace").read()
    return r
