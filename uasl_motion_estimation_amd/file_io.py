"""Frame ingest and configuration.

Mirrors include/MotionEstimation/core/file_IO.h and src/core/file_IO.cpp:
``loadYML`` (:30-98) with the DatasetInfo / FrameInfo / TrackingInfo
structures (file_IO.h:30-141), ``IOFile::openFile`` / ``check_header``
(:100-131), ``ImageFile::readData`` (:133-145) for ``image_data.csv``, and
the image loaders ``loadImage`` / ``loadImages`` (cam{0,1}_image%0Nd[_appendix].png,
:296-364) and ``loadImageKitti`` / ``loadImagesKitti`` (L_/R_ %0Nd .png, rows
0..373, :313-340), and ``ImageReader`` (file_IO.h:300-421) in both its
IMAGES and VIDEO modes -- the latter over ``VideoCapture``, an uncompressed
RIFF-AVI reader (8-bit palettised / 24-bit BGR frames; no codec exists here,
so compressed streams do not open, as cv::VideoCapture without a backend).
``StereoImageStream`` stages frames into pinned host memory and uploads them
asynchronously to HBM for the device pipeline.

Host-side plumbing (like the reference's); no GPU compute.  Image decoding
uses Pillow.  ``cv::imread(..., IMREAD_GRAYSCALE)`` semantics: 8-bit gray is
read as is, 16-bit gray keeps the high byte (libpng strip_16), colour images
use OpenCV's fixed-point BGR2GRAY weights ((4899 R + 9617 G + 1868 B + 8192)
>> 14) -- libpng's own rgb_to_gray rounding in OpenCV's PNG decoder is not
reproducible here, so colour input is "parity unpinned".
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field

import numpy as np

from .rotation_utils import Quat
from .vo import Method, Parameters


# ------------------------------------------------------------------ config
@dataclass
class FrameInfo:
    """file_IO.h:45-68."""
    fframe: int = 0
    lframe: int = 0
    skip: int = 1
    bias_frame: int = 0
    init: int = 0

    def read(self, node: dict):
        self.fframe = _int(node, "start")
        self.lframe = _int(node, "stop")
        self.skip = _int(node, "rate")
        self.bias_frame = _int(node, "bframe")
        self.init = _int(node, "initframe")
        if not self.skip:
            self.skip = 1


@dataclass
class TrackingInfo:
    """file_IO.h:71-96 (a missing feat_cov reads as 0 and becomes 1.0, as in the reference)."""
    nb_feats: int = 500
    window_size: int = 5
    ba_rate: int = 0
    parallax: float = 10.0
    feat_cov: float = 0.25

    def read(self, node: dict):
        self.nb_feats = _int(node, "feats")
        self.window_size = _int(node, "window")
        self.ba_rate = _int(node, "ba_rate")
        self.parallax = _float(node, "parallax")
        self.feat_cov = _float(node, "feat_cov")
        if not self.feat_cov:
            self.feat_cov = 1.0


@dataclass
class DatasetInfo:
    """file_IO.h:99-141.  type: "mono" | "stereo"; poses: "absolute" | "relative"."""
    dir: str = ""
    image_filename: str = ""
    gt_filename: str = ""
    imu_filename: str = ""
    is_video: bool = False
    gps_orientation: float = 0.0
    type: str = "mono"
    scaled_traj: bool = False
    poses: str = "absolute"
    cam_ID: int = 0
    q_init: Quat = field(default_factory=Quat)
    q_cam_to_base: Quat = field(default_factory=Quat)
    p_init: np.ndarray = field(default_factory=lambda: np.zeros(3))
    p_cam_to_base: np.ndarray = field(default_factory=lambda: np.zeros(3))

    def read(self, node: dict):
        self.dir = _str(node, "dir")
        self.image_filename = _str(node, "image_file")
        self.gt_filename = _str(node, "gt_file")
        self.imu_filename = _str(node, "imu_file")
        self.is_video = _str(node, "video") == "true"
        self.gps_orientation = _float(node, "gps")
        self.type = "mono" if _str(node, "type") == "mono" else "stereo"
        self.scaled_traj = _str(node, "scaled") == "true"
        self.poses = "absolute" if _str(node, "poses") == "absolute" else "relative"
        self.cam_ID = _int(node, "camID")
        q = _vec(node, "init_orientation", 4)
        if np.linalg.norm(q) > 0:
            self.q_init = Quat(*q)
        q = _vec(node, "cam_orientation", 4)
        if np.linalg.norm(q) > 0:
            self.q_cam_to_base = Quat(*q)
        self.p_init = _vec(node, "init_position", 3)
        self.p_cam_to_base = _vec(node, "cam_position", 3)


@dataclass
class MonoParameters:
    """MonoVisualOdometry::parameters fields read by loadYML (file_IO.cpp:83-92)."""
    fu: float = 1.0
    fv: float = 1.0
    cu: float = 0.0
    cv: float = 0.0
    ransac: bool = True
    inlier_threshold: float = 2.0
    nb_fixed_frames: int = 2


@dataclass
class Config:
    """The globals loadYML fills (file_IO.cpp:19-27)."""
    dataset_info: DatasetInfo = field(default_factory=DatasetInfo)
    frame_info: FrameInfo = field(default_factory=FrameInfo)
    tracking_info: TrackingInfo = field(default_factory=TrackingInfo)
    param_stereo: Parameters = field(default_factory=Parameters)
    param_mono: MonoParameters = field(default_factory=MonoParameters)
    appendix: str = ""


# cv::FileNode conversions of a missing node: int/double 0, string "", Vec zeros
def _node(node, key):
    return node.get(key) if isinstance(node, dict) else None


def _int(node, key) -> int:
    """(int)FileNode: missing 0, INT as is, REAL cvRound (half-even), anything else INT_MAX."""
    v = _node(node, key)
    if v is None:
        return 0
    if isinstance(v, bool):
        return 0x7FFFFFFF
    if isinstance(v, int):
        return v
    if isinstance(v, float):
        return int(round(v))
    return 0x7FFFFFFF


def _float(node, key) -> float:
    v = _node(node, key)
    if v is None or isinstance(v, (dict, list, str)):
        return 0.0
    return float(v)


def _str(node, key) -> str:
    v = _node(node, key)
    if v is None or isinstance(v, (dict, list)):
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _vec(node, key, n) -> np.ndarray:
    v = _node(node, key)
    if isinstance(v, dict) and "data" in v:  # !!opencv-matrix
        v = v["data"]
    if isinstance(v, list) and len(v) == n:
        return np.asarray(v, np.float64)
    return np.zeros(n)


def _load_filestorage_yaml(path: str) -> dict:
    """cv::FileStorage YAML: a '%YAML:1.0' directive line and '!!opencv-matrix'
    tagged maps; parsed with yaml.SafeLoader (nothing executable)."""
    import yaml

    with open(path) as f:
        text = f.read()
    text = re.sub(r"^%YAML[: ]1\.\d+\s*\n", "", text)
    text = text.replace("!!opencv-matrix", "")

    class _Loader(yaml.SafeLoader):
        pass

    # OpenCV writes 'true' / 'false' as strings; keep scalars as plain strings
    # only for the keys the reader compares as strings (handled by _str).
    data = yaml.load(text, Loader=_Loader)  # noqa: S506 (SafeLoader subclass)
    return data if isinstance(data, dict) else {}


def loadYML(filename: str, cfg: Config | None = None) -> Config | None:
    """bool loadYML(string filename) (file_IO.cpp:30-98): returns the filled
    Config (the reference fills globals), or None when the file cannot be opened."""
    if not os.path.isfile(filename):
        print("YML file could not be opened!")
        return None
    fs = _load_filestorage_yaml(filename)
    cfg = cfg or Config()
    for key, obj in (("dataset", cfg.dataset_info), ("frames", cfg.frame_info), ("tracking", cfg.tracking_info)):
        node = fs.get(key)
        if node is None:  # read(node, x, default): an empty node keeps the default
            continue
        obj.read(node)
    calib = fs.get("calib") or {}
    if cfg.dataset_info.type == "stereo":
        ps = cfg.param_stereo
        ps.fu1 = _float(calib, "f1")
        ps.fu2 = _float(calib, "f2")
        ps.fv1 = _float(calib, "f1")
        ps.fv2 = _float(calib, "f2")
        if not ps.fu1:
            ps.fu1 = _float(calib, "fu1")
            ps.fu2 = _float(calib, "fu2")
            ps.fv1 = _float(calib, "fv1")
            ps.fv2 = _float(calib, "fv2")
        ps.cu1 = _float(calib, "cu") or _float(calib, "cu1")
        ps.cu2 = _float(calib, "cu") or _float(calib, "cu2")
        ps.cv1 = _float(calib, "cv") or _float(calib, "cv1")
        ps.cv2 = _float(calib, "cv") or _float(calib, "cv2")
        ps.baseline = _float(calib, "baseline")
        ps.ransac = _str(calib, "ransac") == "true"
        ps.weighting = _str(calib, "weighting") == "true"
        ps.inlier_threshold = _float(calib, "threshold")
        ps.method = Method.GN if _str(calib, "method") == "GN" else Method.LM
        ps.nb_fixed_frames = _int(calib, "fixed_frames")
    else:
        pm = cfg.param_mono
        pm.fu = _float(calib, "fu")
        pm.fv = _float(calib, "fv")
        if not pm.fu:
            pm.fu = _float(calib, "f")
            pm.fv = _float(calib, "f")
        pm.cu = _float(calib, "cu")
        pm.cv = _float(calib, "cv")
        pm.ransac = bool(_int(calib, "ransac"))
        pm.inlier_threshold = _float(calib, "threshold")
        pm.nb_fixed_frames = _int(calib, "fixed_frames")
    cfg.appendix = _str(fs, "appendix")
    return cfg


# ------------------------------------------------------------------ csv files
class IOFile:
    """IOFile (file_IO.cpp:100-131): a text file whose first line holds a
    '#'-prefixed, comma-separated header."""

    def __init__(self, filename: str = ""):
        self.m_filename = filename
        self.m_file = None
        self.m_file_desc: list[str] = []
        if filename:
            self.openFile(filename)

    def openFile(self, filename: str) -> int:
        self.m_filename = filename
        try:
            self.m_file = open(filename)
        except OSError:
            print(f"could not open file: {filename}")
            self.m_file = None
            return 0
        return self.check_header()

    def is_open(self) -> bool:
        return self.m_file is not None

    def check_header(self) -> int:
        if self.m_file is None:
            return 0
        header = self.m_file.readline().rstrip("\n")
        pos = header.find("#")
        if pos < 0:
            print(f"could not find header in {self.m_filename}")
            self.m_file.close()
            self.m_file = None
            return 0
        buff = ""
        for ch in header[pos + 1:]:
            if ch != ",":
                buff += ch
            elif buff != "":
                self.m_file_desc.append(buff)
                buff = ""
        if buff != "":
            self.m_file_desc.append(buff)
        return 1

    def getFileDesc(self) -> list[str]:
        return list(self.m_file_desc)

    def close(self):
        if self.m_file is not None:
            self.m_file.close()
            self.m_file = None


_IMG_LINE = re.compile(r"^\s*([+-]?\d+)\s*(\S)\s*([+-]?\d+)")


class ImageFile(IOFile):
    """ImageFile::readData (file_IO.cpp:133-145): 'nb<sep>stamp' per line."""

    def readData(self):
        """Returns (ok, nb, stamp) -- ok is 1 on success, 0 at end of file / parse failure."""
        if self.m_file is None:
            return 0, 0, 0
        line = self.m_file.readline()
        if not line:
            return 0, 0, 0
        m = _IMG_LINE.match(line)
        if not m:
            return 0, 0, 0
        return 1, int(m.group(1)), int(m.group(3))


# ------------------------------------------------------------------ images
def imread_gray(path: str) -> np.ndarray | None:
    """cv::imread(path, IMREAD_GRAYSCALE) for PNG: None when unreadable (the reference gets an empty Mat)."""
    from PIL import Image

    try:
        with Image.open(path) as im:
            im.load()
            mode = im.mode
            if mode == "L":
                return np.asarray(im, np.uint8).copy()
            if mode in ("I;16", "I;16B", "I;16L", "I"):
                a = np.asarray(im).astype(np.uint32)
                return (a >> 8).astype(np.uint8)
            if mode == "P":
                im = im.convert("RGB")
                mode = "RGB"
            if mode in ("RGB", "RGBA", "LA"):
                if mode == "LA":
                    return np.asarray(im, np.uint8)[..., 0].copy()
                a = np.asarray(im, np.int32)
                g = (a[..., 0] * 4899 + a[..., 1] * 9617 + a[..., 2] * 1868 + 8192) >> 14
                return g.astype(np.uint8)
            if mode == "1":
                return (np.asarray(im, np.uint8) * 255).astype(np.uint8)
            return np.asarray(im.convert("L"), np.uint8).copy()
    except (OSError, ValueError):
        return None


def _num(nb: int, padding: int) -> str:
    return str(int(nb)).zfill(padding) if nb >= 0 else "-" + str(-int(nb)).zfill(padding - 1)


def _cam_path(directory: str, cam: int, nb: int, padding: int, appendix: str) -> str:
    return f"{directory}/cam{cam}_image{_num(nb, padding)}{('_' + appendix) if appendix else ''}.png"


def loadImage(directory: str, cam_nb: int, img_nb: int, padding: int = 5, appendix: str = ""):
    """cv::Mat loadImage(dir, cam_nb, img_nb, padding) (file_IO.cpp:356-364)."""
    path = _cam_path(directory, cam_nb, img_nb, padding, appendix)
    img = imread_gray(path)
    if img is None:
        print(f"cannot read {path}")
    return img


def loadImages(directory: str, nb: int, padding: int = 5, stereo: bool = True, appendix: str = ""):
    """pair<Mat,Mat> loadImages(dir, nb[, padding]) (file_IO.cpp:296-311, 342-354); the
    second image only for stereo setups (dataset_info.type)."""
    left = loadImage(directory, 0, nb, padding, appendix)
    right = loadImage(directory, 1, nb, padding, appendix) if stereo else None
    return left, right


def _kitti(path: str):
    img = imread_gray(path)
    if img is None:
        print(f"cannot read {path}")
        return None
    return img[0:374]  # rowRange(Range(0, 374))


def loadImageKitti(directory: str, cam_nb: int, img_nb: int, padding: int = 6):
    """cv::Mat loadImageKitti (file_IO.cpp:330-340): always the L_ image, as in the reference."""
    return _kitti(f"{directory}/L_{_num(img_nb, padding)}.png")


def loadImagesKitti(directory: str, nb: int, padding: int = 6, stereo: bool = True):
    """loadImagesKitti (file_IO.cpp:313-328)."""
    left = _kitti(f"{directory}/L_{_num(nb, padding)}.png")
    right = _kitti(f"{directory}/R_{_num(nb, padding)}.png") if stereo else None
    return left, right


# ------------------------------------------------------------------ device staging
class StereoImageStream:
    """Frames of a dataset (image_data.csv + cam{0,1}_image*.png) staged for the
    device pipeline: each pair is copied into a pinned host slot and uploaded
    to HBM with an asynchronous H2D on the context stream (double-buffered,
    so decoding frame k+1 overlaps the device work of frame k).  Yields
    (nb, stamp, dev_left, dev_right, width, height).  Mirrors ImageReader's
    image mode (file_IO.h:300-340): frames before frame_info.fframe are skipped,
    every frame_info.skip-th frame is used, and reading stops after lframe (if > 0)."""

    def __init__(self, cfg: Config, ctx, image_file: str | None = None, padding: int = 5):
        import torch

        self.cfg = cfg
        self.ctx = ctx
        self.padding = padding
        d = cfg.dataset_info.dir
        self.file = ImageFile(image_file or os.path.join(d, cfg.dataset_info.image_filename or "image_data.csv"))
        self._torch = torch
        self._dev = [None, None]
        self._host = [None, None]
        self._slot = 0

    def _ensure(self, shape):
        torch = self._torch
        if self._dev[0] is None or tuple(self._dev[0].shape[1:]) != tuple(shape):
            dev = torch.device("cuda", self.ctx.device)
            self._dev = [torch.empty((2,) + tuple(shape), dtype=torch.uint8, device=dev) for _ in range(2)]
            self._host = [torch.empty((2,) + tuple(shape), dtype=torch.uint8).pin_memory() for _ in range(2)]

    def __iter__(self):
        fi = self.cfg.frame_info
        k = 0
        stereo = self.cfg.dataset_info.type == "stereo"
        while True:
            ok, nb, stamp = self.file.readData()
            if not ok:
                return
            if nb < fi.fframe or (fi.lframe > 0 and nb > fi.lframe):
                if fi.lframe > 0 and nb > fi.lframe:
                    return
                continue
            if (k % max(fi.skip, 1)) != 0:
                k += 1
                continue
            k += 1
            left, right = loadImages(self.cfg.dataset_info.dir, nb, self.padding, stereo, self.cfg.appendix)
            if left is None or (stereo and right is None):
                continue
            right = right if right is not None else left
            self._ensure(left.shape)
            s = self._slot
            self._slot ^= 1
            h = self._host[s]
            h[0].numpy()[...] = left
            h[1].numpy()[...] = right
            stream = self._torch.cuda.ExternalStream(self.ctx.stream_ptr(), device=self.ctx.device)
            with self._torch.cuda.stream(stream):
                self._dev[s].copy_(h, non_blocking=True)
            H, W = left.shape
            yield nb, stamp, self._dev[s][0].data_ptr(), self._dev[s][1].data_ptr(), W, H


# ------------------------------------------------------------------ video (AVI)
CAP_PROP_POS_FRAMES = 1  # cv::CAP_PROP_POS_FRAMES
CAP_PROP_FRAME_WIDTH = 3
CAP_PROP_FRAME_HEIGHT = 4
CAP_PROP_FRAME_COUNT = 7


class VideoCapture:
    """The subset of cv::VideoCapture that ImageReader's VIDEO mode uses
    (file_IO.h:314-316, 366-372, 398-401: open / isOpened / get(CAP_PROP_POS_FRAMES)
    / grab / operator>>), for uncompressed RIFF AVI only: one video stream of
    BI_RGB frames ('00db' / '00dc' chunks), 8-bit palettised or 24-bit BGR, bottom-up
    (positive biHeight) or top-down rows, each row padded to 4 bytes.  There is
    no codec here, so compressed streams (MJPG, H.264, ...) do not open, exactly
    as cv::VideoCapture::open fails without a backend for them: isOpened() is
    False.  Frames come back as OpenCV's default CAP_PROP_CONVERT_RGB output:
    H x W x 3 BGR uint8 (a palettised frame through its palette), rows top-down.
    The file is memory-mapped: frames are decoded when read, never all at once."""

    def __init__(self, filename: str | None = None):
        self._mm = None
        self._frames: list[tuple[int, int]] = []
        self._pos = 0
        self._grabbed = -1
        self.width = self.height = 0
        if filename:
            self.open(filename)

    # --- RIFF walk
    def open(self, filename: str) -> bool:
        import mmap
        import struct

        self.release()
        try:
            with open(filename, "rb") as fh:
                mm = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
        except (OSError, ValueError):
            return False
        try:
            if len(mm) < 12 or mm[0:4] != b"RIFF" or mm[8:12] != b"AVI ":
                raise ValueError("not a RIFF AVI file")
            fmt = None
            vstream = -1
            nstream = 0
            frames: list[tuple[int, int]] = []

            def walk(off: int, end: int, depth: int):
                nonlocal fmt, vstream, nstream
                while off + 8 <= end:
                    cid = bytes(mm[off:off + 4])
                    size = struct.unpack_from("<I", mm, off + 4)[0]
                    body = off + 8
                    if body + size > len(mm):
                        size = len(mm) - body  # truncated file: keep what is there
                    if cid in (b"RIFF", b"LIST"):
                        walk(body + 4, body + size, depth + 1)
                    elif cid == b"strh":
                        typ = bytes(mm[body:body + 4])
                        if typ == b"vids" and vstream < 0:
                            vstream = nstream
                        nstream += 1
                    elif cid == b"strf" and vstream == nstream - 1 and fmt is None:
                        fmt = (body, size)
                    elif len(cid) == 4 and cid[2:4] in (b"db", b"dc") and cid[0:2].isdigit():
                        if vstream >= 0 and int(cid[0:2]) == vstream:
                            frames.append((body, size))
                    off = body + size + (size & 1)

            walk(12, len(mm), 0)
            if fmt is None:
                raise ValueError("no video stream format")
            body, size = fmt
            (_bisz, w, h, _planes, bits, comp, _isz, _xp, _yp, clr_used, _clr_imp) = struct.unpack_from(
                "<IiiHHIIiiII", mm, body)
            if comp not in (0,) or bits not in (8, 24):
                raise ValueError(f"unsupported AVI frame format (compression {comp:#x}, {bits} bits)")
            pal = None
            if bits == 8:
                n = clr_used or 256
                raw = np.frombuffer(mm, np.uint8, count=4 * n, offset=body + _bisz).reshape(n, 4)
                pal = np.zeros((256, 3), np.uint8)
                pal[:n] = raw[:, :3]  # RGBQUAD: B, G, R, reserved
            self._mm = mm
            self._frames = frames
            self._bits = bits
            self._pal = pal
            self.width, self.height = int(w), abs(int(h))
            self._bottom_up = h > 0
            self._stride = ((self.width * bits // 8) + 3) & ~3
            return True
        except (ValueError, struct.error):
            mm.close()
            return False

    def isOpened(self) -> bool:
        return self._mm is not None

    def release(self):
        if self._mm is not None:
            self._mm.close()
        self._mm = None
        self._frames = []
        self._pos = 0
        self._grabbed = -1

    def get(self, prop: int) -> float:
        if self._mm is None:
            return 0.0
        if prop == CAP_PROP_POS_FRAMES:
            return float(self._pos)
        if prop == CAP_PROP_FRAME_COUNT:
            return float(len(self._frames))
        if prop == CAP_PROP_FRAME_WIDTH:
            return float(self.width)
        if prop == CAP_PROP_FRAME_HEIGHT:
            return float(self.height)
        return 0.0

    def grab(self) -> bool:
        if self._mm is None or self._pos >= len(self._frames):
            self._grabbed = -1
            return False
        self._grabbed = self._pos
        self._pos += 1
        return True

    def retrieve(self):
        if self._grabbed < 0:
            return False, None
        off, size = self._frames[self._grabbed]
        w, h, s = self.width, self.height, self._stride
        if size < s * h:  # a dropped / empty frame chunk
            return False, None
        rows = np.frombuffer(self._mm, np.uint8, count=s * h, offset=off).reshape(h, s)
        if self._bottom_up:
            rows = rows[::-1]
        if self._bits == 8:
            img = self._pal[rows[:, :w]]
        else:
            img = rows[:, :3 * w].reshape(h, w, 3).copy()
        return True, np.ascontiguousarray(img)

    def read(self):
        if not self.grab():
            return False, None
        return self.retrieve()


def bgr2gray(img: np.ndarray) -> np.ndarray:
    """cv::cvtColor(COLOR_BGR2GRAY) on 8U: fixed-point (4899 R + 9617 G + 1868 B + 8192) >> 14."""
    c = img.astype(np.int32)
    return ((c[..., 2] * 4899 + c[..., 1] * 9617 + c[..., 0] * 1868 + 8192) >> 14).astype(np.uint8)


class ImageReader:
    """ImageReader (file_IO.h:300-421): the next frame of a dataset, from the PNG
    directory (Type.IMAGES) or from cam{i}_image.avi (Type.VIDEO), frame numbers
    from image_data.csv (ImageFile) when it exists, else advanced by
    frame_info.skip.  The constructor reads until img_nb reaches
    frame_info.fframe, as the reference does; readStereo / readMono return
    (left, right) / an image, or empty (None) where the reference returns an
    empty Mat.  A video frame is seeked by grabbing until CAP_PROP_POS_FRAMES
    reaches img_nb, then read and converted to gray when it has 3 channels."""

    class Type:
        IMAGES = 0
        VIDEO = 1

    def __init__(self, cfg: Config, filename: str = "", type_: int = 0, padding: int = 5):
        self.cfg = cfg
        self.padding = padding
        self.fimage = ImageFile(filename)
        stereo = cfg.dataset_info.type == "stereo"
        self.cap = [VideoCapture() for _ in range(2 if stereo else 1)]
        self.type = type_
        self.img_nb = 0
        self.img_stamp = 0
        if not self.fimage.is_open():
            print(f"[ImageReader] warning: could not find an image file in {cfg.dataset_info.dir}")
        if self.type == ImageReader.Type.VIDEO:
            self._open_video()
        self._seek_first()

    def _open_video(self):
        for i, c in enumerate(self.cap):
            c.open(f"{self.cfg.dataset_info.dir}/cam{i}_image.avi")

    def _seek_first(self):
        # do { readMono(); } while (img_nb < fframe).  The reference spins for
        # ever once image_data.csv runs out before fframe (readData fails and
        # img_nb stops moving); here the loop ends there instead.
        while True:
            self._last_ok = True
            self.readMono()
            if not (self.img_nb < self.cfg.frame_info.fframe) or not self._last_ok:
                break

    def openReader(self, filename: str = "", type_: int = 0):
        self.fimage = ImageFile(filename or f"{self.cfg.dataset_info.dir}/image_data.csv")
        self.type = type_
        if not self.fimage.is_open():
            print(f"[ImageReader] warning: could not find an image file in {self.cfg.dataset_info.dir}")
        elif self.type == ImageReader.Type.VIDEO:
            self._open_video()
        self._seek_first()

    def isValid(self) -> bool:
        valid = bool(self.img_nb)
        if self.type == ImageReader.Type.VIDEO:
            for c in self.cap:
                valid = valid or c.isOpened()  # (the reference's ||, kept)
        return valid

    def get_img_nb(self) -> int:
        return self.img_nb

    def _advance(self) -> bool:
        if self.fimage.is_open():
            for _ in range(self.cfg.frame_info.skip):
                ok, nb, stamp = self.fimage.readData()
                if not ok:
                    print(f"[Error] could not read image{self.img_nb} in {self.cfg.dataset_info.dir}")
                    self._last_ok = False
                    return False
                self.img_nb, self.img_stamp = nb, stamp
        else:
            self.img_nb += self.cfg.frame_info.skip
        return True

    def _video_frame(self, c: VideoCapture):
        while c.get(CAP_PROP_POS_FRAMES) < self.img_nb:
            if not c.grab():
                break
        ok, img = c.read()
        if not ok:
            return None
        return bgr2gray(img) if img.ndim == 3 else img

    def readStereo(self):
        if not self._advance():
            return None, None
        if self.type == ImageReader.Type.IMAGES:
            return loadImages(self.cfg.dataset_info.dir, self.img_nb, self.padding, True, self.cfg.appendix)
        if len(self.cap) < 2 or not self.cap[0].isOpened() or not self.cap[1].isOpened():
            print("[ImageReader] Warning: video stream is not opened!")
            return None, None
        return self._video_frame(self.cap[0]), self._video_frame(self.cap[1])

    def readMono(self):
        if not self._advance():
            return None
        if self.type == ImageReader.Type.IMAGES:
            return loadImage(self.cfg.dataset_info.dir, self.cfg.dataset_info.cam_ID, self.img_nb, self.padding,
                             self.cfg.appendix)
        if not self.cap[0].isOpened():
            print("[ImageReader] Warning: video stream is not opened!")
            return None
        return self._video_frame(self.cap[0])
