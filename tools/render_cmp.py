import sys; sys.path.insert(0,'/root/repo')
import numpy as np, torch
from uasl_motion_estimation_amd import synthetic as S
K, fr = S.corridor_frames_torch(S.SEED0+5, 1280, 720, 200, 2, device='cuda')
sc, K2, ref = S.stereo_stream(S.SEED0+5, 1280, 720, 2, first_id=200, scene_kind='corridor')
for k in range(2):
    L = fr[k][0].cpu().numpy(); R = fr[k][1].cpu().numpy()
    print('gpu vs numpy: left equal', (L == ref[k].left).mean(), 'right', (R == ref[k].right).mean(), np.abs(L.astype(int)-ref[k].left).max())
