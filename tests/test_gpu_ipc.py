"""IPC collectives (one-shot / two-shot all-reduce, direct all-gather) kernel (``ops/csrc/ipc_allreduce.hip``) with 2 and 3 processes sharing
the box's GPU: handle exchange, per-block epoch barriers, slot reuse, bitwise rank-order sums."""
import pytest

from ._dist import run_distributed

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nprocs", [2, 3])
def test_ipc_allreduce(gpu, nprocs):
    run_distributed("tests.ipc_checks:check_ipc_allreduce", nprocs, timeout=110, keep_gpu=True)


def test_ipc_through_communication(gpu):
    run_distributed("tests.ipc_checks:check_ipc_through_communication", 2, timeout=110, keep_gpu=True,
                    env_extra={"HEAT_IPC_ALLREDUCE": "1"})


def test_ipc_timeout_is_loud(gpu):
    run_distributed("tests.ipc_checks:check_ipc_timeout_is_loud", 2, timeout=110, keep_gpu=True)


@pytest.mark.parametrize("nprocs", [2, 3])
def test_ipc_allgather_two_shot(gpu, nprocs):
    run_distributed("tests.ipc_checks:check_ipc_allgather_and_two_shot", nprocs, timeout=110, keep_gpu=True)


@pytest.mark.parametrize("nprocs", [2, 3])
def test_ipc_halo(gpu, nprocs):
    run_distributed("tests.ipc_checks:check_ipc_halo", nprocs, timeout=110, keep_gpu=True,
                    env_extra={"HEAT_IPC_ALLREDUCE": "1"})


def test_ipc_iterative_paths(gpu):
    run_distributed("tests.ipc_checks:check_ipc_iterative_paths", 2, timeout=110, keep_gpu=True,
                    env_extra={"HEAT_IPC_ALLREDUCE": "1"})
