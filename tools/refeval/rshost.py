"""Host objects for rsinterp: rav1e's frame / region types, re-expressed over
flat Python lists so the reference's own function text can run on them.

These are data-model restatements, not the code under test:
  Plane / PlaneConfig / PlaneSlice      src/frame/plane.rs:22-47, 316-342, 480-590
  PlaneRegion(Mut), Rect, Area          src/tiling/plane_region.rs:18-105, 136-260,
                                        342-358, 440-600
  BlockSize (enum order, width/height)  src/partition.rs:116-140, 179-215
  MotionVector, FilterMode              src/mc.rs:28-66
"""
from rsinterp import RangeV, Slice, Struct, StructType, TInt, wrap

BLOCK_NAMES = ["4X4", "4X8", "8X4", "8X8", "8X16", "16X8", "16X16", "16X32", "32X16",
               "32X32", "32X64", "64X32", "64X64", "64X128", "128X64", "128X128",
               "4X16", "16X4", "8X32", "32X8", "16X64", "64X16"]


class BlockSizeV(int):
    """A BlockSize enum value (its discriminant is the table index)."""

    def __new__(cls, idx):
        o = int.__new__(cls, idx)
        w, h = BLOCK_NAMES[idx].split("X")
        o.w, o.h = int(w), int(h)
        return o

    def width(self):
        return TInt(self.w, "usize")

    def height(self):
        return TInt(self.h, "usize")

    def width_log2(self):
        return TInt(self.w.bit_length() - 1, "usize")

    def height_log2(self):
        return TInt(self.h.bit_length() - 1, "usize")

    def area(self):
        return TInt(self.w * self.h, "usize")

    def width_mi(self):
        return TInt(self.w >> 2, "usize")

    def height_mi(self):
        return TInt(self.h >> 2, "usize")

    def largest_chroma_tx_size(self, xdec, ydec):
        """src/partition.rs:288-297: subsampled_size -> max_txsize_rect_lookup
        -> av1_get_coded_tx_size (a 64-point dimension codes as 32)."""
        w = max(4, self.w >> int(xdec))
        h = max(4, self.h >> int(ydec))
        return TxDims(min(w, 32), min(h, 32))


class TxDims:
    """A TxSize by its dimensions (width_mi / height_mi, src/transform/mod.rs)."""

    def __init__(self, w, h):
        self.w, self.h = w, h

    def width_mi(self):
        return TInt(self.w >> 2, "usize")

    def height_mi(self):
        return TInt(self.h >> 2, "usize")


class _BlockSizeNS:
    def __init__(self):
        for i, n in enumerate(BLOCK_NAMES):
            setattr(self, "BLOCK_" + n, BlockSizeV(i))
        self.BLOCK_SIZES_ALL = TInt(22, "usize")

    def from_width_and_height(self, w, h):
        return BlockSizeV(BLOCK_NAMES.index("%dX%d" % (int(w), int(h))))


BlockSize = _BlockSizeNS()


class PlaneConfig:
    def __init__(self, width, height, xdec, ydec, xpad, ypad, bytes_per_px=1):
        # src/frame/plane.rs:52-75 (Plane::new geometry)
        xorigin_align = max(1, 32 // bytes_per_px)
        self.width, self.height = width, height
        self.xdec, self.ydec = xdec, ydec
        self.xpad, self.ypad = xpad, ypad
        self.xorigin = (xpad + xorigin_align - 1) // xorigin_align * xorigin_align
        self.yorigin = ypad
        stride = self.xorigin + width + xpad
        self.stride = (stride + xorigin_align - 1) // xorigin_align * xorigin_align
        self.alloc_height = self.yorigin + height + ypad

    def __getattribute__(self, k):
        v = object.__getattribute__(self, k)
        return TInt(v, "usize") if isinstance(v, int) and not isinstance(v, TInt) else v


class Plane:
    """A padded plane; `data` is the flat allocation (stride × alloc_height)."""

    def __init__(self, cfg, data):
        self.cfg = cfg
        assert len(data) == cfg.stride * cfg.alloc_height
        self.data = data

    @classmethod
    def from_full(cls, full, xorigin, yorigin, width, height, xdec=0, ydec=0, bpp=1):
        """Wrap a (alloc_height, stride) array laid out like Plane::new."""
        cfg = PlaneConfig.__new__(PlaneConfig)
        cfg.width, cfg.height, cfg.xdec, cfg.ydec = width, height, xdec, ydec
        cfg.xorigin, cfg.yorigin = xorigin, yorigin
        cfg.stride, cfg.alloc_height = full.shape[1], full.shape[0]
        cfg.xpad, cfg.ypad = xorigin, yorigin
        return cls(cfg, [int(v) for v in full.reshape(-1)])

    # src/frame/plane.rs:316-322
    def slice(self, po):
        return PlaneSlice(self, int(po.x), int(po.y))

    mut_slice = slice

    # src/frame/plane.rs:178-187
    def region(self, area):
        rect = to_rect(area, self.cfg.xdec, self.cfg.ydec, self.cfg.stride - self.cfg.xorigin,
                       self.cfg.alloc_height - self.cfg.yorigin)
        return PlaneRegion(self, rect)

    region_mut = region

    def as_region(self):
        return self.region(Struct("Area::StartingAt", {"x": 0, "y": 0}))

    as_region_mut = as_region

    def _row_range(self, x, y):  # src/frame/plane.rs:335-343
        base_y = self.cfg.yorigin + int(y)
        base_x = self.cfg.xorigin + int(x)
        assert base_y >= 0 and base_x >= 0
        base = base_y * self.cfg.stride + base_x
        return base, base + self.cfg.stride - base_x

    def row_range(self, x, y):  # as the reference's callers see it: a Range<usize>
        from rsinterp import RangeV
        a, b = self._row_range(x, y)
        return RangeV(TInt(a, "usize"), TInt(b, "usize"), False)

    def p(self, x, y):  # src/frame/plane.rs PlaneSlice::p via the plane
        return self.data[self._row_range(x, y)[0]]


class PlaneSlice:
    """src/frame/plane.rs:480-590."""

    def __init__(self, plane, x, y):
        self.plane, self.x, self.y = plane, x, y

    def index_row(self, r):
        a, b = self.plane._row_range(self.x, self.y + r)
        return Slice(self.plane.data, a, b)

    def clamp(self):
        c = self.plane.cfg
        return PlaneSlice(self.plane, max(min(self.x, c.width), -c.xorigin),
                          max(min(self.y, c.height), -c.yorigin))

    def subslice(self, xo, yo):
        return PlaneSlice(self.plane, self.x + int(xo), self.y + int(yo))

    def reslice(self, xo, yo):
        return PlaneSlice(self.plane, self.x + int(xo), self.y + int(yo))

    def go_up(self, i):
        return PlaneSlice(self.plane, self.x, self.y - int(i))

    def go_left(self, i):
        return PlaneSlice(self.plane, self.x - int(i), self.y)

    def p(self, x, y):  # src/frame/plane.rs:548-553
        return self.plane.p(self.x + int(x), self.y + int(y))

    def as_ptr(self):
        from rsinterp import Ptr
        return Ptr(self.plane.data, self.plane._row_range(self.x, self.y)[0])


def to_rect(area, xdec, ydec, parent_w, parent_h):
    """Area::to_rect, src/tiling/plane_region.rs:74-105 (pixel variants)."""
    kind = area._name.split("::")[-1]
    f = area._f
    if kind == "Rect":
        return Struct("Rect", {"x": wrap(f["x"], "isize"), "y": wrap(f["y"], "isize"),
                               "width": wrap(f["width"], "usize"),
                               "height": wrap(f["height"], "usize")})
    if kind == "StartingAt":
        x, y = int(f["x"]), int(f["y"])
        return Struct("Rect", {"x": wrap(x, "isize"), "y": wrap(y, "isize"),
                               "width": wrap(parent_w - x, "usize"),
                               "height": wrap(parent_h - y, "usize")})
    raise NotImplementedError("Area::" + kind)


class PlaneRegion:
    """src/tiling/plane_region.rs:110-600 (PlaneRegion and PlaneRegionMut)."""

    def __init__(self, plane, rect, origin=None):
        c = plane.cfg
        self.plane = plane
        self.plane_cfg = c
        self._rect = rect
        if origin is None:
            assert rect.x >= -c.xorigin and rect.y >= -c.yorigin
            assert c.xorigin + rect.x + rect.width <= c.stride
            assert c.yorigin + rect.y + rect.height <= c.alloc_height
            origin = (c.yorigin + rect.y) * c.stride + c.xorigin + rect.x
        self.origin = int(origin)

    def rect(self):
        return self._rect

    def data_ptr(self):
        from rsinterp import Ptr
        return Ptr(self.plane.data, self.origin)

    data_ptr_mut = data_ptr

    def index_row(self, r):  # Index<usize>, :342-358
        assert 0 <= r < self._rect.height, "row %d of %d" % (r, self._rect.height)
        a = self.origin + r * self.plane_cfg.stride
        return Slice(self.plane.data, a, a + int(self._rect.width))

    def rows_iter(self):
        from rsinterp import It
        return It(self.index_row(r) for r in range(int(self._rect.height)))

    rows_iter_mut = rows_iter

    def subregion(self, area):  # :229-255
        rect = to_rect(area, self.plane_cfg.xdec, self.plane_cfg.ydec, int(self._rect.width),
                       int(self._rect.height))
        assert 0 <= rect.x <= self._rect.width and 0 <= rect.y <= self._rect.height
        origin = self.origin + int(rect.y) * self.plane_cfg.stride + int(rect.x)
        ab = Struct("Rect", {"x": wrap(self._rect.x + rect.x, "isize"),
                             "y": wrap(self._rect.y + rect.y, "isize"),
                             "width": rect.width, "height": rect.height})
        return PlaneRegion(self.plane, ab, origin)

    subregion_mut = subregion

    def as_const(self):
        return self

    def vert_windows(self, h):  # :175-187, 534-566
        from rsinterp import It
        h = int(h)
        n = max(0, int(self._rect.height) - h + 1)

        def gen():
            for k in range(n):
                rect = Struct("Rect", {"x": self._rect.x, "y": wrap(self._rect.y + k, "isize"),
                                       "width": self._rect.width, "height": wrap(h, "usize")})
                yield PlaneRegion(self.plane, rect, self.origin + k * self.plane_cfg.stride)
        return It(gen())

    def horz_windows(self, w):  # :189-201, 568-600
        from rsinterp import It
        w = int(w)
        n = max(0, int(self._rect.width) - w + 1)

        def gen():
            for k in range(n):
                rect = Struct("Rect", {"x": wrap(self._rect.x + k, "isize"), "y": self._rect.y,
                                       "width": wrap(w, "usize"), "height": self._rect.height})
                yield PlaneRegion(self.plane, rect, self.origin + k)
        return It(gen())


def motion_vector(row, col):
    return Struct("MotionVector", {"row": wrap(row, "i16"), "col": wrap(col, "i16")})


class _MVType(StructType):
    def __init__(self):
        super().__init__("MotionVector", {"row": "i16", "col": "i16"})

    def default(self):
        return motion_vector(0, 0)


class _FilterMode:
    REGULAR, SMOOTH, SHARP, BILINEAR, SWITCHABLE = (TInt(i, "usize") for i in range(5))


class _Cpu:
    RUST = TInt(0, "usize")

    def as_index(self):
        return 0


def base_env():
    """Names every loaded reference function may refer to."""
    return {
        "BlockSize": BlockSize,
        "MotionVector": _MVType(),
        "FilterMode": _FilterMode(),
        "CpuFeatureLevel": _Cpu(),
        "Area": StructType("Area"),
        "Rect": StructType("Rect", {"x": "isize", "y": "isize", "width": "usize",
                                    "height": "usize"}),
        "PlaneOffset": StructType("PlaneOffset", {"x": "isize", "y": "isize"}),
        "Range": RangeV,
    }
