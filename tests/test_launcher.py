"""``python -m heat_amd.run`` (the mpirun replacement) on CPU/gloo."""
import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, body, n=2):
    script = tmp_path / "prog.py"
    script.write_text(textwrap.dedent(body))
    env = dict(os.environ, PYTHONPATH=REPO, HEAT_COMM_BACKEND="gloo", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    return subprocess.run([sys.executable, "-m", "heat_amd.run", "-n", str(n), "--backend", "gloo", str(script)],
                          capture_output=True, text=True, env=env, timeout=300, cwd=REPO)


def test_launch_two_ranks(tmp_path):
    res = _run(tmp_path, """
        import heat_amd as ht
        x = ht.arange(10, split=0)
        print("SUM", int(ht.sum(x).item()), ht.MPI_WORLD.rank, ht.MPI_WORLD.size)
    """)
    assert res.returncode == 0, res.stderr
    assert "[0] SUM 45 0 2" in res.stdout and "[1] SUM 45 1 2" in res.stdout


def test_launch_failure_propagates(tmp_path):
    res = _run(tmp_path, """
        import sys, heat_amd as ht
        if ht.MPI_WORLD.rank == 1:
            sys.exit(3)
        ht.MPI_WORLD.Barrier()
    """)
    assert res.returncode != 0
