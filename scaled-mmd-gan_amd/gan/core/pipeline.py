"""Input pipelines of gan/core/pipeline.py for the BASELINE datasets, feeding
HBM-resident batches to the trainer.

* ``Cifar10`` (pipeline.py:383-410): ``data_batch_1..5`` + ``test_batch`` of
  the CIFAR-10 python distribution (pickled dicts; the binary distribution's
  ``data_batch_*.bin`` / ``test_batch.bin`` are read too, with no pickle), all
  10 classes, /255, shuffled once with numpy seed 547, then served in order as
  a cyclic queue (``tf.train.input_producer(shuffle=False).dequeue_many``).
  The whole set (60000 x 3 x 32 x 32 fp32, 737 MB) is copied to HBM once and
  a batch is a slice of it: no host work per step.
* ``ImagenetDataFlow`` (:170-207) / ``CelebADataFlow`` (:209-248): TFRecord
  shards ``tf_records_train/train-*`` of ``tf.train.Example`` records with an
  ``image/encoded`` JPEG.  Records are framed and parsed here without
  TensorFlow, JPEGs are decoded by PIL on a pool of host threads (PIL drops
  the GIL), one uint8 batch is copied to the GPU, and the /255 + TF-1.x
  ``resize_bilinear`` (legacy mapping, align_corners=False) run there.
  ImageNet: 256x256x3 -> output_size.  CelebA: crop-or-pad to 178 x 178
  (centred), random left-right flip, random 160 x 160 crop, -> output_size.
  The reference's RecordInput shuffles with seed 301 over a 4000-record
  buffer; here shard order and a 4000-record buffer are shuffled with
  ``numpy.random.default_rng(301)`` (same distribution, not the same order).
* ``Synthetic``: U[0,1] images (the pipelines' value range, :201, :403).

``get_pipeline(dataset)`` mirrors pipeline.py:458-476.
"""
from __future__ import annotations

import glob
import os
import pickle
import queue
import struct
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

# ---------------------------------------------------------------------------
# TFRecord framing: u64 length, u32 masked crc32c(length), data, u32 masked
# crc32c(data) -- all little-endian.
# ---------------------------------------------------------------------------
_CRC_TABLE = []


def crc32c(data: bytes) -> int:
    """CRC-32C (Castagnoli, reflected polynomial 0x82F63B78)."""
    if not _CRC_TABLE:
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            _CRC_TABLE.append(c)
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def read_tfrecords(path, verify=False):
    """Yield the payload of every record of one TFRecord file."""
    with open(path, 'rb') as f:
        while True:
            hdr = f.read(12)
            if not hdr:
                return
            if len(hdr) < 12:
                raise ValueError('%s: truncated record header' % path)
            n, lcrc = struct.unpack('<QI', hdr)
            data = f.read(n)
            tail = f.read(4)
            if len(data) < n or len(tail) < 4:
                raise ValueError('%s: truncated record' % path)
            if verify:
                if masked_crc32c(hdr[:8]) != lcrc:
                    raise ValueError('%s: length crc mismatch' % path)
                if masked_crc32c(data) != struct.unpack('<I', tail)[0]:
                    raise ValueError('%s: data crc mismatch' % path)
            yield data


def write_tfrecords(path, records):
    with open(path, 'wb') as f:
        for data in records:
            ln = struct.pack('<Q', len(data))
            f.write(ln + struct.pack('<I', masked_crc32c(ln)) + data +
                    struct.pack('<I', masked_crc32c(data)))


# ---------------------------------------------------------------------------
# tf.train.Example in protobuf wire format:
#   Example{Features features=1}  Features{map<string,Feature> feature=1}
#   Feature{oneof: BytesList bytes_list=1 | FloatList float_list=2 |
#           Int64List int64_list=3}, each {repeated value=1} (numbers packed)
# ---------------------------------------------------------------------------
def _varint(buf, i):
    r, s = 0, 0
    while True:
        b = buf[i]
        i += 1
        r |= (b & 0x7F) << s
        if b < 0x80:
            return r, i
        s += 7


def _fields(buf):
    """(field number, wire type, value) of a message: an int for varints,
    bytes for length-delimited and fixed-width fields."""
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = bytes(buf[i:i + ln])
            i += ln
        elif wt == 5:
            v = bytes(buf[i:i + 4])
            i += 4
        elif wt == 1:
            v = bytes(buf[i:i + 8])
            i += 8
        else:
            raise ValueError('unsupported protobuf wire type %d' % wt)
        yield fn, wt, v


def _signed64(v):
    return v - (1 << 64) if v >= (1 << 63) else v


def _feature_values(feature):
    vals = []
    for kind, _, lst in _fields(feature):
        for fn, wt, v in _fields(lst):
            if fn != 1:
                continue
            if kind == 1:                                   # bytes_list
                vals.append(v)
            elif kind == 2:                                 # float_list
                vals.extend(np.frombuffer(v, '<f4').tolist() if wt == 2
                            else [struct.unpack('<f', v)[0]])
            elif kind == 3:                                 # int64_list
                if wt == 2:
                    j = 0
                    while j < len(v):
                        x, j = _varint(v, j)
                        vals.append(_signed64(x))
                else:
                    vals.append(_signed64(v))
    return vals


def parse_example(buf):
    """tf.parse_single_example without a schema: {name: list of bytes/int/float}."""
    out = {}
    for fn, _, feats in _fields(buf):
        if fn != 1:
            continue
        for fn2, _, entry in _fields(feats):
            if fn2 != 1:
                continue
            key, feature = None, b''
            for fn3, _, v in _fields(entry):
                if fn3 == 1:
                    key = v.decode()
                elif fn3 == 2:
                    feature = v
            out[key] = _feature_values(feature)
    return out


def _enc_varint(x):
    x &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _enc_field(fn, payload):
    return _enc_varint((fn << 3) | 2) + _enc_varint(len(payload)) + payload


def encode_example(features):
    """tf.train.Example bytes of {name: bytes | int | float | list of one kind}."""
    entries = b''
    for k, v in features.items():
        vals = list(v) if isinstance(v, (list, tuple)) else [v]
        if all(isinstance(x, (bytes, bytearray)) for x in vals):
            feat = _enc_field(1, b''.join(_enc_field(1, bytes(x)) for x in vals))
        elif all(isinstance(x, int) for x in vals):
            feat = _enc_field(3, _enc_field(1, b''.join(_enc_varint(x) for x in vals)))
        else:
            feat = _enc_field(2, _enc_field(1, np.asarray(vals, '<f4').tobytes()))
        entries += _enc_field(1, _enc_field(1, k.encode()) + _enc_field(2, feat))
    return _enc_field(1, entries)


# ---------------------------------------------------------------------------
# image ops with TF-1.x semantics
# ---------------------------------------------------------------------------
def _legacy_axis(in_size, out_size, device):
    """tf.image.resize_bilinear (align_corners=False, legacy scaler):
    in = out * (in_size / out_size) in fp32; lower = floor(in),
    upper = min(lower + 1, in_size - 1), lerp = in - lower."""
    scale = np.float32(in_size) / np.float32(out_size)
    pos = np.arange(out_size, dtype=np.float32) * scale
    lo = np.floor(pos).astype(np.int64)
    hi = np.minimum(lo + 1, in_size - 1)
    lerp = (pos - lo.astype(np.float32)).astype(np.float32)
    return (torch.from_numpy(lo).to(device), torch.from_numpy(hi).to(device),
            torch.from_numpy(lerp).to(device))


def resize_bilinear_tf(x, out_h, out_w):
    """x [B, H, W, C] float32 -> [B, out_h, out_w, C] as TF-1.x resize_bilinear:
    top = tl + (tr - tl) * xl; bottom = bl + (br - bl) * xl;
    out = top + (bottom - top) * yl."""
    _, H, W, _ = x.shape
    y0, y1, yl = _legacy_axis(H, out_h, x.device)
    x0, x1, xl = _legacy_axis(W, out_w, x.device)
    top, bot = x[:, y0], x[:, y1]
    xl = xl.view(1, 1, -1, 1)
    t = top[:, :, x0] + (top[:, :, x1] - top[:, :, x0]) * xl
    b = bot[:, :, x0] + (bot[:, :, x1] - bot[:, :, x0]) * xl
    return t + (b - t) * yl.view(1, -1, 1, 1)


def crop_or_pad(img, th, tw):
    """tf.image.resize_image_with_crop_or_pad of an HWC array (centred)."""
    h, w = img.shape[:2]
    oy, ox = max((h - th) // 2, 0), max((w - tw) // 2, 0)
    img = img[oy:oy + min(h, th), ox:ox + min(w, tw)]
    h, w = img.shape[:2]
    if h == th and w == tw:
        return img
    out = np.zeros((th, tw) + img.shape[2:], img.dtype)
    py, px = (th - h) // 2, (tw - w) // 2
    out[py:py + h, px:px + w] = img
    return out


def decode_jpeg(buf, channels=3):
    """tf.image.decode_jpeg(channels=c) -> HWC uint8."""
    import io
    from PIL import Image
    im = Image.open(io.BytesIO(buf)).convert('RGB' if channels == 3 else 'L')
    a = np.asarray(im, dtype=np.uint8)
    return a if a.ndim == 3 else a[:, :, None]


# ---------------------------------------------------------------------------
# pipelines
# ---------------------------------------------------------------------------
class Pipeline:
    """Base: ``next()`` returns one [batch, c, s, s] fp32 tensor on ``device``.
    With ``world`` > 1 data-parallel replicas, replica ``rank`` draws its own
    batches (the reference's towers each dequeue their own, model.py:187-216)."""

    def __init__(self, output_size, c_dim, batch_size, data_dir, device=None, rank=0, world=1):
        self.output_size = output_size
        self.c_dim = c_dim
        self.batch_size = batch_size
        self.data_dir = data_dir
        self.rank, self.world = rank, world
        if device is None:
            device = (torch.device('cuda', torch.cuda.current_device())
                      if torch.cuda.is_available() else torch.device('cpu'))
        self.device = torch.device(device)

    def next(self):
        raise NotImplementedError

    def stop(self):
        pass


class Synthetic(Pipeline):
    def __init__(self, *args, seed=0, **kwargs):
        super().__init__(*args, **kwargs)
        self.gen = torch.Generator(device=self.device).manual_seed(seed + self.rank)

    def next(self):
        s = self.output_size
        return torch.rand(self.batch_size, self.c_dim, s, s, device=self.device,
                          generator=self.gen)


def _cifar_file(data_dir, name):
    """(uint8 [n, 3, 32, 32], labels) of one CIFAR-10 batch: the python
    distribution's pickled dict (misc.unpickle), else the binary one's .bin
    (1 label byte + 3072 pixel bytes per image)."""
    p = os.path.join(data_dir, name)
    if os.path.exists(p):
        with open(p, 'rb') as f:
            d = pickle.load(f, encoding='latin1')
        d = {(k.decode() if isinstance(k, bytes) else k): v for k, v in d.items()}
        return (np.asarray(d['data'], np.uint8).reshape(-1, 3, 32, 32),
                np.asarray(d['labels'], np.int64))
    raw = np.fromfile(p + '.bin', np.uint8).reshape(-1, 1 + 3 * 32 * 32)
    return raw[:, 1:].reshape(-1, 3, 32, 32), raw[:, 0].astype(np.int64)


class Cifar10(Pipeline):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        categories = np.arange(10)
        xs = []
        for name in ['data_batch_%d' % b for b in range(1, 6)] + ['test_batch']:
            x, y = _cifar_file(self.data_dir, name)
            xs.append(x[np.isin(y, categories)])
        X = np.concatenate(xs, 0).astype(np.float32) / 255.
        np.random.seed(547)                                 # pipeline.py:405-407
        np.random.shuffle(X)
        self.data = torch.from_numpy(X).to(self.device)     # resident in HBM
        self.pos = self.rank * self.batch_size              # replicas interleave batches

    def next(self):
        n, b = self.data.shape[0], self.batch_size
        p = self.pos % n
        if p + b <= n:
            out = self.data[p:p + b]
        else:                                               # the queue wraps around
            out = torch.cat([self.data[p:], self.data[:p + b - n]], 0)
        self.pos = (p + self.world * b) % n
        return out


class DataFlow(Pipeline):
    """TFRecord shards -> decoded uint8 batches on a host thread (``prefetch``
    batches ahead) -> GPU: /255, resize, NCHW."""
    regex = 'tf_records_train/train-*'
    buffer_size = 4000

    def __init__(self, *args, workers=16, prefetch=3, seed=301, verify=False, **kwargs):
        super().__init__(*args, **kwargs)
        files = sorted(glob.glob(os.path.join(self.data_dir, self.regex)))
        if not files:
            raise FileNotFoundError('no TFRecord shards match %s'
                                    % os.path.join(self.data_dir, self.regex))
        # replicas read disjoint shards when there are enough of them
        self.files = files[self.rank::self.world] if len(files) >= self.world else files
        self.rng = np.random.default_rng(seed + self.rank)
        self.verify = verify
        self.pool = ThreadPoolExecutor(max_workers=workers)
        self.q = queue.Queue(maxsize=prefetch)
        self._stop = threading.Event()
        self._err = None
        self.thread = threading.Thread(target=self._produce, daemon=True)
        self.thread.start()

    def _records(self):
        """Endless shuffled stream: shards in random order each pass, records
        through a shuffle buffer of ``buffer_size``."""
        buf = []
        while True:
            for i in self.rng.permutation(len(self.files)):
                for rec in read_tfrecords(self.files[i], self.verify):
                    buf.append(rec)
                    if len(buf) >= self.buffer_size:
                        j = int(self.rng.integers(len(buf)))
                        buf[j], buf[-1] = buf[-1], buf[j]
                        yield buf.pop()
                if self._stop.is_set():
                    return

    def _produce(self):
        try:
            recs = self._records()
            while not self._stop.is_set():
                batch = [next(recs) for _ in range(self.batch_size)]
                seeds = self.rng.integers(0, 2 ** 31, size=len(batch))
                imgs = list(self.pool.map(self._decode, batch, seeds))
                arr = np.stack(imgs, 0)
                while not self._stop.is_set():
                    try:
                        self.q.put(arr, timeout=0.1)
                        break
                    except queue.Full:
                        pass
        except BaseException as e:          # surfaced by next()
            if not self._stop.is_set():
                self._err = e
                self.q.put(None)

    def _decode(self, rec, seed):
        ex = parse_example(rec)
        img = decode_jpeg(ex['image/encoded'][0], self.c_dim)
        return self.preprocess_host(img, np.random.default_rng(seed))

    def preprocess_host(self, img, rng):
        return img

    def next(self):
        arr = self.q.get()
        if arr is None:
            raise RuntimeError('input pipeline failed') from self._err
        x = torch.from_numpy(arr)
        if self.device.type == 'cuda':
            x = x.pin_memory()
        x = x.to(self.device, non_blocking=True).float() / 255.
        s = self.output_size
        return resize_bilinear_tf(x, s, s).permute(0, 3, 1, 2).contiguous()

    def stop(self):
        self._stop.set()
        self.thread.join(timeout=5.0)
        self.pool.shutdown(wait=False)


class ImagenetDataFlow(DataFlow):
    """pipeline.py:175-207: decode, reshape [256, 256, 3], /255, resize."""

    def preprocess_host(self, img, rng):
        if img.shape[:2] != (256, 256):
            raise ValueError('imagenet records hold 256x256 JPEGs (pipeline.py:199), got %s'
                             % (img.shape,))
        return img


class CelebADataFlow(DataFlow):
    """pipeline.py:214-248: crop-or-pad to 178, random flip, random 160 crop."""
    base_size = 160
    random_crop = 9

    def preprocess_host(self, img, rng):
        bs = self.base_size + 2 * self.random_crop
        img = crop_or_pad(img, bs, bs)
        if self.random_crop > 0:
            if rng.random() < 0.5:
                img = img[:, ::-1]
            oy, ox = rng.integers(0, bs - self.base_size + 1, size=2)
            img = img[oy:oy + self.base_size, ox:ox + self.base_size]
        return np.ascontiguousarray(img)


def get_pipeline(dataset):
    """pipeline.py:458-476 (lsun / mnist / GaussianMix are outside this build)."""
    table = {'celebA': CelebADataFlow, 'cifar10': Cifar10, 'imagenet': ImagenetDataFlow,
             'synthetic': Synthetic}
    if dataset not in table:
        raise ValueError('invalid dataset: %s' % dataset)
    return table[dataset]
