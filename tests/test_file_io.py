"""Frame ingest and configuration (src/core/file_IO.cpp:30-145, 296-364).
Fixtures are written here (PNG via Pillow, a FileStorage-style YAML, an
image_data.csv); expected values follow the reference's code paths,
including its quirks (f1 read into fu1 and fv1, missing feat_cov -> 1.0,
rate 0 -> 1, KITTI rows 0..373).  Colour-PNG conversion (libpng inside
OpenCV) is parity unpinned; gray 8/16-bit are exact."""
import numpy as np
import pytest

from uasl_motion_estimation_amd import file_io as F


YML = """%YAML:1.0
dataset:
   dir: "{dir}"
   image_file: image_data.csv
   type: stereo
   video: "false"
   poses: relative
   camID: 1
   init_orientation: [ 0.0, 0.0, 0.0, 0.0 ]
   cam_orientation: [ 0.5, 0.5, 0.5, 0.5 ]
   cam_position: [ 1.0, 2.0, 3.0 ]
frames:
   start: 2
   stop: 6
   rate: 0
tracking:
   feats: 2000
   window: 20
   parallax: 7.5
calib:
   f1: 1152.0
   f2: 1150.0
   cu: 640.0
   cv1: 360.0
   cv2: 361.0
   baseline: 0.5
   ransac: "true"
   threshold: 2.0
   method: GN
   fixed_frames: 2
appendix: rect
"""


def test_loadYML_reference_semantics(tmp_path):
    p = tmp_path / "cfg.yml"
    p.write_text(YML.format(dir=str(tmp_path)))
    cfg = F.loadYML(str(p))
    d, fr, tr, ps = cfg.dataset_info, cfg.frame_info, cfg.tracking_info, cfg.param_stereo
    assert d.type == "stereo" and d.poses == "relative" and d.cam_ID == 1 and not d.is_video
    assert np.allclose(d.q_init.coeffs(), [1, 0, 0, 0])          # zero quaternion: keeps identity
    assert np.allclose(d.q_cam_to_base.coeffs(), [0.5, 0.5, 0.5, 0.5])
    assert np.allclose(d.p_cam_to_base, [1, 2, 3]) and np.allclose(d.p_init, 0)
    assert (fr.fframe, fr.lframe, fr.skip) == (2, 6, 1)           # rate 0 -> 1
    assert (tr.nb_feats, tr.window_size, tr.parallax, tr.feat_cov) == (2000, 20, 7.5, 1.0)  # missing feat_cov -> 1
    assert ps.fu1 == ps.fv1 == 1152.0 and ps.fu2 == ps.fv2 == 1150.0  # f1 read into fu1 AND fv1
    assert ps.cu1 == ps.cu2 == 640.0 and (ps.cv1, ps.cv2) == (360.0, 361.0)
    assert ps.baseline == 0.5 and ps.ransac and ps.inlier_threshold == 2.0 and ps.nb_fixed_frames == 2
    assert cfg.appendix == "rect"
    assert F.loadYML(str(tmp_path / "missing.yml")) is None


def test_image_file_header_and_rows(tmp_path):
    p = tmp_path / "image_data.csv"
    p.write_text("# img_nb, timestamp,,extra\n3,1000\n4 , 2000\n5;3000\nbad\n")
    f = F.ImageFile(str(p))
    assert f.getFileDesc() == [" img_nb", " timestamp", "extra"]
    assert f.readData() == (1, 3, 1000)
    assert f.readData() == (1, 4, 2000)
    assert f.readData() == (1, 5, 3000)  # any single separator character
    assert f.readData()[0] == 0
    q = tmp_path / "noheader.csv"
    q.write_text("1,2\n")
    assert F.IOFile().openFile(str(q)) == 0


def test_image_loaders(tmp_path):
    from PIL import Image

    rng = np.random.default_rng(0)
    g8 = rng.integers(0, 256, (400, 64), dtype=np.uint8)
    g16 = rng.integers(0, 65536, (30, 20), dtype=np.uint16)
    rgb = rng.integers(0, 256, (10, 12, 3), dtype=np.uint8)
    Image.fromarray(g8).save(tmp_path / "cam0_image00007_rect.png")
    Image.fromarray(g8[::-1].copy()).save(tmp_path / "cam1_image00007_rect.png")
    Image.fromarray(g16).save(tmp_path / "g16.png")
    Image.fromarray(rgb).save(tmp_path / "rgb.png")
    Image.fromarray(g8).save(tmp_path / "L_000042.png")
    Image.fromarray(g8[::-1].copy()).save(tmp_path / "R_000042.png")
    L, R = F.loadImages(str(tmp_path), 7, appendix="rect")
    assert np.array_equal(L, g8) and np.array_equal(R, g8[::-1])
    assert np.array_equal(F.imread_gray(str(tmp_path / "g16.png")), (g16 >> 8).astype(np.uint8))
    c = rgb.astype(np.int64)
    exp = ((c[..., 0] * 4899 + c[..., 1] * 9617 + c[..., 2] * 1868 + 8192) >> 14).astype(np.uint8)
    assert np.array_equal(F.imread_gray(str(tmp_path / "rgb.png")), exp)
    kl, kr = F.loadImagesKitti(str(tmp_path), 42)
    assert kl.shape == (374, 64) and np.array_equal(kl, g8[:374]) and np.array_equal(kr, g8[::-1][:374])
    assert F.loadImage(str(tmp_path), 0, 8) is None  # missing file: empty Mat


@pytest.mark.gpu
def test_stereo_stream_stages_frames_on_the_device(tmp_path, ctx):
    """Pinned staging + async H2D on the context stream; the device copies are the files' pixels."""
    from PIL import Image

    rng = np.random.default_rng(1)
    frames = {}
    for nb in range(2, 9):
        L = rng.integers(0, 256, (48, 64), dtype=np.uint8)
        R = rng.integers(0, 256, (48, 64), dtype=np.uint8)
        Image.fromarray(L).save(tmp_path / f"cam0_image{nb:05d}_rect.png")
        Image.fromarray(R).save(tmp_path / f"cam1_image{nb:05d}_rect.png")
        frames[nb] = (L, R)
    (tmp_path / "image_data.csv").write_text("#img,stamp\n" + "".join(f"{nb},{nb * 100}\n" for nb in range(2, 9)))
    (tmp_path / "cfg.yml").write_text(YML.format(dir=str(tmp_path)))
    cfg = F.loadYML(str(tmp_path / "cfg.yml"))
    seen = []
    for nb, stamp, dL, dR, W, H in F.StereoImageStream(cfg, ctx):
        gotL = np.zeros((H, W), np.uint8)
        gotR = np.zeros((H, W), np.uint8)
        ctx.synchronize()
        ctx.d2h(gotL, dL)
        ctx.d2h(gotR, dR)
        assert np.array_equal(gotL, frames[nb][0]) and np.array_equal(gotR, frames[nb][1]) and stamp == 100 * nb
        seen.append(nb)
    assert seen == [2, 3, 4, 5, 6]  # frames.start .. frames.stop


AVI_DIR = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "avi")


def test_video_capture_reads_committed_avi():
    """Uncompressed RIFF AVI (file_IO.h:305-343's cv::VideoCapture, VIDEO mode): the committed
    fixtures (tests/golden/make_avi.py, an independent RIFF writer) decode to their frames bit for bit --
    8-bit palettised bottom-up rows with padding, JUNK / odd-sized chunks, and 24-bit BGR top-down."""
    import os

    exp = np.load(os.path.join(AVI_DIR, "frames.npz"))
    cap = F.VideoCapture(os.path.join(AVI_DIR, "cam0_image.avi"))
    assert cap.isOpened() and cap.get(F.CAP_PROP_FRAME_COUNT) == 5
    assert (cap.get(F.CAP_PROP_FRAME_WIDTH), cap.get(F.CAP_PROP_FRAME_HEIGHT)) == (20, 12)
    for k in range(5):
        assert cap.get(F.CAP_PROP_POS_FRAMES) == k
        ok, img = cap.read()
        assert ok and img.shape == (12, 20, 3)
        assert np.array_equal(F.bgr2gray(img), exp["cam0"][k])  # gray palette -> BGR -> gray is exact
    ok, img = cap.read()
    assert not ok and img is None  # end of stream
    c = F.VideoCapture(os.path.join(AVI_DIR, "bgr24.avi"))
    for k in range(3):
        ok, img = c.read()
        assert ok and np.array_equal(img, exp["bgr24"][k])
    # not an AVI / missing file: not opened (cv::VideoCapture::open fails)
    assert not F.VideoCapture(os.path.join(AVI_DIR, "image_data.csv")).isOpened()
    assert not F.VideoCapture(os.path.join(AVI_DIR, "missing.avi")).isOpened()


def test_video_capture_rejects_compressed_stream(tmp_path):
    import os

    data = bytearray(open(os.path.join(AVI_DIR, "bgr24.avi"), "rb").read())
    i = data.find(b"strf")
    data[i + 8 + 16:i + 8 + 20] = b"MJPG"  # biCompression
    p = tmp_path / "mjpg.avi"
    p.write_bytes(bytes(data))
    assert not F.VideoCapture(str(p)).isOpened()


def test_image_reader_video_mode():
    """ImageReader(Type::VIDEO) (file_IO.h:300-421): the constructor reads until img_nb reaches
    frames.start (frame numbers from image_data.csv), readStereo seeks each stream by grabbing to
    CAP_PROP_POS_FRAMES == img_nb and returns the gray frames; past the CSV's end the pair is empty."""
    import os

    exp = np.load(os.path.join(AVI_DIR, "frames.npz"))
    cfg = F.Config()
    cfg.dataset_info.dir = AVI_DIR
    cfg.dataset_info.type = "stereo"
    cfg.frame_info.fframe = 2
    r = F.ImageReader(cfg, os.path.join(AVI_DIR, "image_data.csv"), F.ImageReader.Type.VIDEO)
    assert r.isValid() and r.get_img_nb() == 2 and r.img_stamp == 1080
    for nb in (3, 4):
        L, R = r.readStereo()
        assert r.get_img_nb() == nb
        assert np.array_equal(L, exp["cam0"][nb]) and np.array_equal(R, exp["cam1"][nb])
    L, R = r.readStereo()
    assert L is None and R is None
    cfg.dataset_info.type = "mono"
    cfg.frame_info.fframe = 0
    cfg.frame_info.skip = 2
    m = F.ImageReader(cfg, os.path.join(AVI_DIR, "image_data.csv"), F.ImageReader.Type.VIDEO)
    assert m.get_img_nb() == 1  # first readMono consumed rows 0 and 1 (skip 2)
    assert np.array_equal(m.readMono(), exp["cam0"][3])
