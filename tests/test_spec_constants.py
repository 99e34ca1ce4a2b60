"""The written specs the oracle and the device share must use the same constants:
a drift would still pass every oracle-vs-numpy CPU test and only show up as GPU parity failures.
Read from the sources (CPU, no build)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _src(*p):
    return open(os.path.join(ROOT, *p)).read()


def test_ata_block_spec_shared():
    """A^T A of the LSQ fits: ORC_ATA_BLOCK-point blocks, 64 blocks per superblock (oracle)
    == kAtaBlock-point blocks, 64 per superblock (kernels_nonmin.hip)."""
    oc = _src("oracle", "usac_oracle.c")
    dev = _src("ransac_amd", "csrc", "kernels_nonmin.hip")
    ob = int(re.search(r"#define ORC_ATA_BLOCK (\d+)u", oc).group(1))
    osup = re.search(r"#define ORC_ATA_SUPER \((\d+)u \* ORC_ATA_BLOCK\)", oc)
    db = int(re.search(r"constexpr uint32_t kAtaBlock = (\d+);", dev).group(1))
    assert ob == db == 16
    assert osup and int(osup.group(1)) == 64
    assert "64 * kAtaBlock" in dev  # the device superblock: 64 blocks (one lane each)
    assert oc.count("ORC_ATA_SUPER) {") + oc.count("ORC_ATA_SUPER < n") >= 4  # both fits use it


def test_guarded_essential_band():
    """The guarded essential residual's band (kernels_fund.hip) is 2^-16 of thr on both sides and
    the timed-kernel parity bound in bench.py carries its c thr 2^-18 term."""
    f = _src("ransac_amd", "csrc", "kernels_fund.hip")
    assert "thr * 0.9999847412109375f" in f and "thr * 1.0000152587890625f" in f
    assert 0.9999847412109375 == 1 - 2.0 ** -16 and 1.0000152587890625 == 1 + 2.0 ** -16
    b = _src("bench.py")
    assert "bound += cnt * thr * 2.0 ** -18" in b
