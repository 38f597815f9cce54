"""Reading the channel count RCCL opened per communicator from its INFO init log
(utils/rccl_log.py; bench.py records it at N > 1)."""
from distributed_pytorch_training_amd.utils import rccl_log

# two communicators initialised one after the other in one process (torch's, then the framework's),
# with the library's own format strings (librccl.so: "%s comm %p rank %d nranks %d ... - Init COMPLETE")
LOG = """\
host:1:1 [0] NCCL INFO ncclCommInitRankConfig comm 0x55d0c0000010 rank 0 nranks 8 cudaDev 0 nvmlDev 0 busId 5000 commId 0x1 - Init START
host:1:1 [0] NCCL INFO Channel 00/32 :    0   1   2   3   4   5   6   7
host:1:1 [0] NCCL INFO Channel 31/32 :    0   7   6   5   4   3   2   1
host:1:1 [0] NCCL INFO 32 coll channels, 0 collnet channels, 0 nvls channels, 32 p2p channels, 4 p2p channels per peer
host:1:1 [0] NCCL INFO ncclCommInitRankConfig comm 0x55d0c0000010 rank 0 nranks 8 cudaDev 0 nvmlDev 0 busId 5000 commId 0x1 - Init COMPLETE
host:1:1 [0] NCCL INFO ncclCommInitRank comm 0x55d0c0abcdef rank 0 nranks 8 cudaDev 0 nvmlDev 0 busId 5000 commId 0x2 - Init START
host:1:1 [0] NCCL INFO Channel 00/16 :    0   1   2   3   4   5   6   7
host:1:1 [0] NCCL INFO 16 coll channels, 0 collnet channels, 0 nvls channels, 16 p2p channels, 2 p2p channels per peer
host:1:1 [0] NCCL INFO ncclCommInitRank comm 0x55d0c0abcdef rank 0 nranks 8 cudaDev 0 nvmlDev 0 busId 5000 parent (nil) splitCount 0 color 0 key 0 - Init COMPLETE
"""


def test_channels_keyed_by_communicator():
    got = rccl_log.channels_by_comm(LOG)
    assert got[0x55d0c0000010] == {"coll_channels": 32, "rank": 0, "nranks": 8}
    assert got[0x55d0c0abcdef]["coll_channels"] == 16


def test_ring_lines_are_the_fallback():
    text = "\n".join(l for l in LOG.splitlines() if "coll channels" not in l)
    assert rccl_log.channels_by_comm(text)[0x55d0c0000010]["coll_channels"] == 32


def test_opened_channels_reads_this_process_file(tmp_path):
    import os
    prefix = str(tmp_path / "rccl")
    env = rccl_log.debug_env(prefix)
    assert env["NCCL_DEBUG"] == "INFO" and env["NCCL_DEBUG_FILE"].endswith(".%p.log")
    (tmp_path / f"rccl.{os.getpid()}.log").write_text(LOG)
    assert rccl_log.opened_channels(0x55d0c0abcdef, prefix) == 16
    assert rccl_log.opened_channels(0x1234, prefix) is None
    assert rccl_log.opened_channels(0x1234, str(tmp_path / "missing")) is None
