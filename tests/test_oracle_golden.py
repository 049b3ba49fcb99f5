"""The oracle reproduces its committed golden fixtures, and decodes the synthetic
captures to the frame numbers / CLV time codes the generator wrote."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle.capture import FMT_BY_EXT
from oracle.framer import decode_capture

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, 'golden')


def load_case(case):
    import sys
    sys.path.insert(0, GOLD)
    import make_golden
    with open(os.path.join(GOLD, case + '.json')) as fh:
        return make_golden, json.load(fh)


@pytest.mark.parametrize('case', ['ntsc_cav_u8_0p2s', 'ntsc_clv_u8_0p2s', 'ntsc_cav_r30_0p15s', 'ntsc_cav_lds_0p15s',
                                  'pal_clv_u8_0p2s', 'pal_clv_lds_0p15s',
                                  'ntsc_cav_s16_0p15s', 'ntsc_cav_u8_mid_0p2s'])
def test_oracle_matches_golden(case):
    mg, gold = load_case(case)
    data = mg.build_capture(case)
    assert hashlib.sha256(data).hexdigest() == gold['capture_sha256']
    c = mg.CASES[case]
    frames, pcm, meta = decode_capture(data, FMT_BY_EXT[c['fmt']], system=c['system'])
    assert len(frames) == len(gold['frames'])
    for f, a, m, g in zip(frames, pcm, meta, gold['frames']):
        assert hashlib.sha256(f.tobytes()).hexdigest() == g['tbc_sha256']
        assert hashlib.sha256(a.tobytes()).hexdigest() == g['pcm_sha256']
        assert m == g['meta']
    if frames and 'comb_rgb48_sha256' in gold['frames'][0]:
        from oracle.comb import Comb2D
        rgb = Comb2D().process(np.stack(frames))
        assert [hashlib.sha256(r.tobytes()).hexdigest() for r in rgb] == \
            [g['comb_rgb48_sha256'] for g in gold['frames']]


def test_synthetic_vbi_frame_numbers():
    _, gold = load_case('ntsc_cav_u8_0p2s')
    nrs = [g['meta']['vbi']['framenr'] for g in gold['frames']]
    assert nrs == list(range(nrs[0], nrs[0] + len(nrs)))
    _, gold = load_case('ntsc_clv_u8_0p2s')
    nrs = [g['meta']['vbi']['framenr'] for g in gold['frames']]
    assert nrs == [5400, 5401, 5402, 5403]
    assert all(g['meta']['vbi']['isclv'] for g in gold['frames'])
