"""Input pipelines and checkpoint files on CPU (gan/core/pipeline.py against
gan/core/pipeline.py of the reference, TFRecord / tf.train.Example formats,
TF-1.x resize_bilinear).  All data here is synthetic, written by the tests."""
import io
import os
import pickle
import struct

import numpy as np
import pytest

torch = pytest.importorskip('torch')

from gan.core import pipeline as P  # noqa: E402


def test_crc32c_known_answer():
    # RFC 3720 B.4 check value of "123456789"
    assert P.crc32c(b'123456789') == 0xE3069283
    assert P.crc32c(b'') == 0


def test_example_roundtrip():
    feats = {'image/encoded': b'\xff\xd8jpeg bytes\x00', 'image/height': 256,
             'image/class/label': -3, 'image/format': b'JPEG', 'f': [0.5, -2.25]}
    ex = P.parse_example(P.encode_example(feats))
    assert ex['image/encoded'] == [b'\xff\xd8jpeg bytes\x00']
    assert ex['image/height'] == [256] and ex['image/class/label'] == [-3]
    assert ex['image/format'] == [b'JPEG'] and ex['f'] == [0.5, -2.25]


def test_tfrecord_framing(tmp_path):
    recs = [b'a' * n for n in (0, 1, 300, 70000)]
    path = str(tmp_path / 'x.tfrecord')
    P.write_tfrecords(path, recs)
    assert list(P.read_tfrecords(path, verify=True)) == recs
    raw = bytearray(open(path, 'rb').read())
    raw[12 + 0 + 4 + 12] ^= 1                          # flip a bit of record 1's payload
    open(path, 'wb').write(bytes(raw))
    with pytest.raises(ValueError):
        list(P.read_tfrecords(path, verify=True))


def _resize_ref(x, oh, ow):
    """Plain-loop restatement of TF-1.x resize_bilinear (legacy scaler),
    tensorflow/core/kernels/resize_bilinear_op.cc, in float32."""
    B, H, W, C = x.shape
    hs, ws = np.float32(H) / np.float32(oh), np.float32(W) / np.float32(ow)
    out = np.zeros((B, oh, ow, C), np.float32)
    for y in range(oh):
        iy = np.float32(y) * hs
        y0 = int(np.floor(iy))
        y1 = min(y0 + 1, H - 1)
        yl = np.float32(iy - np.float32(y0))
        for xx in range(ow):
            ix = np.float32(xx) * ws
            x0 = int(np.floor(ix))
            x1 = min(x0 + 1, W - 1)
            xl = np.float32(ix - np.float32(x0))
            t = x[:, y0, x0] + (x[:, y0, x1] - x[:, y0, x0]) * xl
            b = x[:, y1, x0] + (x[:, y1, x1] - x[:, y1, x0]) * xl
            out[:, y, xx] = t + (b - t) * yl
    return out


@pytest.mark.parametrize('hw,ohw', [((256, 256), (64, 64)), ((160, 160), (64, 64)),
                                    ((7, 9), (5, 13)), ((32, 32), (32, 32))])
def test_resize_bilinear_tf(hw, ohw):
    rng = np.random.default_rng(0)
    x = rng.random((2,) + hw + (3,)).astype(np.float32)
    got = P.resize_bilinear_tf(torch.tensor(x), *ohw).numpy()
    np.testing.assert_allclose(got, _resize_ref(x, *ohw), rtol=0, atol=1e-6)
    if hw == (256, 256):                               # scale 4: exact samples
        np.testing.assert_array_equal(got, x[:, ::4, ::4])


def test_crop_or_pad():
    img = np.arange(218 * 178 * 3, dtype=np.int64).reshape(218, 178, 3)
    out = P.crop_or_pad(img, 178, 178)                 # CelebA aligned: crop 20 rows each side
    np.testing.assert_array_equal(out, img[20:198])
    small = np.ones((10, 6, 1), np.uint8)
    out = P.crop_or_pad(small, 14, 8)
    assert out.shape == (14, 8, 1) and out.sum() == 60 and out[2:12, 1:7].all()


def _jpeg(arr):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format='JPEG', quality=95)
    return b.getvalue()


def _shards(root, n_shards, per_shard, hw, seed=0):
    rng = np.random.default_rng(seed)
    d = root / 'tf_records_train'
    d.mkdir()
    imgs = []
    for s in range(n_shards):
        recs = []
        for _ in range(per_shard):
            a = rng.integers(0, 256, size=hw + (3,), dtype=np.uint8)
            imgs.append(a)
            recs.append(P.encode_example({'image/encoded': _jpeg(a), 'image/height': hw[0],
                                          'image/width': hw[1], 'image/format': b'JPEG'}))
        P.write_tfrecords(str(d / ('train-%05d-of-%05d' % (s, n_shards))), recs)
    return imgs


def test_imagenet_dataflow(tmp_path):
    _shards(tmp_path, 2, 5, (256, 256))
    P.DataFlow.buffer_size = 4
    try:
        pipe = P.ImagenetDataFlow(64, 3, 6, str(tmp_path), device='cpu', workers=4, verify=True)
        xs = [pipe.next() for _ in range(3)]
        pipe.stop()
    finally:
        P.DataFlow.buffer_size = 4000
    for x in xs:
        assert x.shape == (6, 3, 64, 64) and x.dtype == torch.float32
        assert 0.0 <= float(x.min()) and float(x.max()) <= 1.0
    # every image is one of the decoded records, resized: check one directly
    from PIL import Image
    a = np.asarray(Image.open(io.BytesIO(_jpeg(np.zeros((256, 256, 3), np.uint8)))))
    assert a.shape == (256, 256, 3)


def test_celeba_preprocess():
    pipe = P.CelebADataFlow.__new__(P.CelebADataFlow)
    img = np.random.default_rng(1).integers(0, 256, (218, 178, 3), dtype=np.uint8)
    outs = [pipe.preprocess_host(img, np.random.default_rng(s)) for s in range(20)]
    assert all(o.shape == (160, 160, 3) for o in outs)
    centre = P.crop_or_pad(img, 178, 178)
    for o in outs:                                     # a 160 crop of the (flipped) centre
        found = False
        for src in (centre, centre[:, ::-1]):
            for oy in range(19):
                for ox in range(19):
                    if np.array_equal(src[oy:oy + 160, ox:ox + 160], o):
                        found = True
                        break
                if found:
                    break
            if found:
                break
        assert found


def test_cifar10_python_and_binary(tmp_path):
    rng = np.random.default_rng(2)
    data = {}
    for name in ['data_batch_%d' % b for b in range(1, 6)] + ['test_batch']:
        x = rng.integers(0, 256, (7, 3072), dtype=np.uint8)
        y = rng.integers(0, 10, 7)
        data[name] = (x, y)
    pyd, bind = tmp_path / 'py', tmp_path / 'bin'
    pyd.mkdir()
    bind.mkdir()
    for name, (x, y) in data.items():
        with open(pyd / name, 'wb') as f:             # the python distribution's format
            pickle.dump({b'data': x, b'labels': list(map(int, y))}, f, protocol=2)
        with open(bind / (name + '.bin'), 'wb') as f:
            f.write(np.concatenate([y.astype(np.uint8)[:, None], x], 1).tobytes())
    a = P.Cifar10(32, 3, 16, str(pyd), device='cpu')
    b = P.Cifar10(32, 3, 16, str(bind), device='cpu')
    torch.testing.assert_close(a.data, b.data, rtol=0, atol=0)
    X = np.concatenate([x for x, _ in data.values()]).reshape(-1, 3, 32, 32)
    X = X.astype(np.float32) / 255.
    np.random.seed(547)
    np.random.shuffle(X)
    np.testing.assert_array_equal(a.data.numpy(), X)
    n = X.shape[0]                                     # 42: batches wrap around the queue
    got = torch.cat([a.next() for _ in range(3)]).numpy()
    np.testing.assert_array_equal(got, np.concatenate([X, X])[:48])
    # two replicas interleave batches
    r0 = P.Cifar10(32, 3, 4, str(bind), device='cpu', rank=0, world=2)
    r1 = P.Cifar10(32, 3, 4, str(bind), device='cpu', rank=1, world=2)
    np.testing.assert_array_equal(r0.next().numpy(), X[0:4])
    np.testing.assert_array_equal(r1.next().numpy(), X[4:8])
    np.testing.assert_array_equal(r0.next().numpy(), X[8:12])
    assert n == 42


def test_make_pipeline_synthetic_only_when_asked(tmp_path):
    from gan.main import make_flags, make_pipeline
    f = make_flags(argv=['-dataset', 'synthetic', '-data_dir', str(tmp_path), '-batch_size', '4'])
    f.real_batch_size = 4
    pipe = make_pipeline(f, 16, 3, torch.device('cpu'))
    assert isinstance(pipe, P.Synthetic)
    x = pipe.next()
    assert x.shape == (4, 3, 16, 16) and 0 <= float(x.min()) and float(x.max()) <= 1


def test_make_pipeline_raises_instead_of_substituting(tmp_path):
    """No silent noise (reference pipeline.py:458-476 raises): absent shards,
    a typo in -dataset, malformed records."""
    from gan.main import make_flags, make_pipeline
    f = make_flags(argv=['-dataset', 'imagenet', '-data_dir', str(tmp_path), '-batch_size', '4'])
    f.real_batch_size = 4
    with pytest.raises(FileNotFoundError):
        make_pipeline(f, 16, 3, torch.device('cpu'))
    f.dataset = 'imagnet'
    with pytest.raises(ValueError, match='invalid dataset'):
        make_pipeline(f, 16, 3, torch.device('cpu'))
    f.dataset = 'cifar10'
    with pytest.raises((FileNotFoundError, ValueError, OSError)):
        make_pipeline(f, 32, 3, torch.device('cpu'))
    # a shard that is not a TFRecord file
    shard_dir = tmp_path / 'tf_records_train'
    shard_dir.mkdir()
    (shard_dir / 'train-00000-of-00001').write_bytes(b'\x01\x02\x03')
    f.dataset = 'imagenet'
    with pytest.raises((ValueError, RuntimeError)):
        pipe = make_pipeline(f, 16, 3, torch.device('cpu'))
        try:
            pipe.next()
        finally:
            pipe.stop()
