"""PoseExpNet forward (posenet/posenet.py:21-96) — torch fp32 CPU restatement (test
infrastructure only, see oracle/__init__.py).

  conv(i, o, k)   Conv2d(k, stride 2, padding (k-1)//2) + ReLU          posenet.py:7-11
  upconv(i, o)    ConvTranspose2d(k 4, stride 2, padding 1) + ReLU      posenet.py:14-18
  forward         cat([target, *refs]) -> conv1 (k7) .. conv7 -> pose_pred (1x1) ->
                  0.01 * spatial mean -> [B, nb_ref, 6]; with output_exp the upconv chain,
                  each output cropped to the matching encoder size, and sigmoid masks
                  (posenet.py:64-96)
Pinned by tests/golden/posenet.npz (the reference module run on seeded weights and inputs).
"""
import torch
import torch.nn.functional as F


def _conv(sd, name, x, k):
    return F.relu(F.conv2d(x, sd[name + ".0.weight"], sd[name + ".0.bias"], stride=2, padding=(k - 1) // 2))


def _upconv(sd, name, x):
    return F.relu(F.conv_transpose2d(x, sd[name + ".0.weight"], sd[name + ".0.bias"], stride=2, padding=1))


def forward(sd, target, refs, output_exp=False):
    """-> (pose [B, nb_ref, 6], [mask1, mask2, mask3, mask4] or None)."""
    nref = len(refs)
    x = torch.cat([target, *refs], 1)
    c1 = _conv(sd, "conv1", x, 7)
    c2 = _conv(sd, "conv2", c1, 5)
    c3 = _conv(sd, "conv3", c2, 3)
    c4 = _conv(sd, "conv4", c3, 3)
    c5 = _conv(sd, "conv5", c4, 3)
    c6 = _conv(sd, "conv6", c5, 3)
    c7 = _conv(sd, "conv7", c6, 3)
    pose = F.conv2d(c7, sd["pose_pred.weight"], sd["pose_pred.bias"])
    pose = 0.01 * pose.mean(3).mean(2).view(pose.size(0), nref, 6)
    if not output_exp:
        return pose, None
    u5 = _upconv(sd, "upconv5", c5)[:, :, :c4.size(2), :c4.size(3)]
    u4 = _upconv(sd, "upconv4", u5)[:, :, :c3.size(2), :c3.size(3)]
    u3 = _upconv(sd, "upconv3", u4)[:, :, :c2.size(2), :c2.size(3)]
    u2 = _upconv(sd, "upconv2", u3)[:, :, :c1.size(2), :c1.size(3)]
    u1 = _upconv(sd, "upconv1", u2)[:, :, :x.size(2), :x.size(3)]
    m = [torch.sigmoid(F.conv2d(u, sd[f"predict_mask{i}.weight"], sd[f"predict_mask{i}.bias"], padding=1))
         for i, u in ((1, u1), (2, u2), (3, u3), (4, u4))]
    return pose, m
