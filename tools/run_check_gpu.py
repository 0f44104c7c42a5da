"""Run one multi-process check of tests/*_checks.py with device buffers (ranks sharing the GPU,
gloo control plane, as tests/test_gpu_dist.py does) and write each rank's FULL output to
gpurun_out/check_<name>_r<rank>.txt. Usage: python tools/run_check_gpu.py tests.dist_checks check_linalg [n]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests._dist import _free_port  # noqa: E402
from tests.test_gpu_dist import ENV  # noqa: E402

mod, name = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 2
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
port = _free_port()
procs = []
for r in range(n):
    env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HEAT_COMM_BACKEND="gloo", OMP_NUM_THREADS="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), **ENV)
    procs.append(subprocess.Popen([sys.executable, "-m", "tests._dist_runner", "{}:{}".format(mod, name)], cwd=ROOT,
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
rc = 0
for r, p in enumerate(procs):
    out, _ = p.communicate(timeout=300)
    with open(os.path.join(ROOT, "gpurun_out", "check_{}_r{}.txt".format(name, r)), "wb") as f:
        f.write(out)
    rc |= p.returncode
print("rc", rc)
sys.exit(1 if rc else 0)
