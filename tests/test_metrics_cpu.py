"""CPU: ground-truth mask decoding of process_dataset (compute_metrics.py:60-61 reads masks with
cv2.imread(IMREAD_GRAYSCALE) > 128): 16-bit PNGs scale by >> 8 and colour PNGs use cv2's BT.601
fixed-point weights (cv2 itself is absent here, so the weights are the published ones, unpinned)."""
import numpy as np
from PIL import Image


def test_read_gray_u8_16bit_and_rgb(tmp_path):
    from s3od_amd.metrics import read_gray_u8
    a = np.array([[0, 32768, 65535, 33000, 32767]], np.uint16)
    Image.fromarray(a).save(tmp_path / "a.png")
    assert read_gray_u8(tmp_path / "a.png").tolist() == [[0, 128, 255, 128, 127]]
    b = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [129, 129, 129]]], np.uint8)
    Image.fromarray(b).save(tmp_path / "b.png")
    assert read_gray_u8(tmp_path / "b.png").tolist() == [[76, 150, 29, 129]]
    g = np.array([[0, 128, 129, 255]], np.uint8)
    Image.fromarray(g).save(tmp_path / "g.png")
    assert (read_gray_u8(tmp_path / "g.png") > 128).tolist() == [[False, False, True, True]]
