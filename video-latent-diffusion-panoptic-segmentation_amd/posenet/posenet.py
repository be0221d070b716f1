"""Drop-in ``PoseExpNet`` for posenet/posenet.py:21-96 (SfMLearner pose / explainability net) on
the gfx950 HIP library — BASELINE config 5's pose network.

Same constructor, module tree and parameter names (``conv1.0.weight`` … ``pose_pred.bias``,
``upconv5.0.weight`` …, ``predict_mask1.weight`` …) and the same ``forward(target_image,
ref_imgs)`` returns as the reference, so its checkpoints load unchanged.  The arithmetic:

  input concat     [target || refs] NCHW -> NHWC, 3 (1 + nb_ref) channels zero-padded to 16,
                   one ldm_nchw_to_nhwc gather (the concat is never materialised)
  conv1..conv7     ldm_conv2d implicit GEMM, k = 7 / 5 / 3, stride 2, padding (k - 1) // 2,
                   ReLU in the epilogue
  pose_pred        1x1 ldm_conv2d (fp32 out); 0.01 * spatial mean -> [B, nb_ref, 6]
  upconv5..1       ConvTranspose2d(k 4, s 2, p 1) as a 3x3 conv with one output group per phase
                   (dy, dx) and the pixel-shuffle epilogue, ReLU; cropped to the encoder size
                   (a no-op whenever the frame size is a multiple of 128)
  predict_mask*    3x3 ldm_conv2d with the sigmoid epilogue, written straight to NCHW fp32

Compute dtype follows the parameters' dtype (fp32: exact-fp32 MFMA; bf16: bf16 MFMA, fp32
accumulate).  No CPU fallback: every op raises if the HIP library is missing.
"""
import torch
import torch.nn as nn
from torch.nn.init import xavier_uniform_, zeros_

from ldmseg.ops import native as K


def conv(in_planes, out_planes, kernel_size=3):                    # posenet.py:7-11
    return nn.Sequential(
        nn.Conv2d(in_planes, out_planes, kernel_size=kernel_size, padding=(kernel_size - 1) // 2, stride=2),
        nn.ReLU(inplace=True))


def upconv(in_planes, out_planes):                                  # posenet.py:14-18
    return nn.Sequential(nn.ConvTranspose2d(in_planes, out_planes, kernel_size=4, stride=2, padding=1),
                         nn.ReLU(inplace=True))


class PoseExpNet(nn.Module):
    def __init__(self, nb_ref_imgs=2, output_exp=False):
        super().__init__()
        self.nb_ref_imgs = nb_ref_imgs
        self.output_exp = output_exp
        conv_planes = [16, 32, 64, 128, 256, 256, 256]
        self.conv1 = conv(3 * (1 + self.nb_ref_imgs), conv_planes[0], kernel_size=7)
        self.conv2 = conv(conv_planes[0], conv_planes[1], kernel_size=5)
        self.conv3 = conv(conv_planes[1], conv_planes[2])
        self.conv4 = conv(conv_planes[2], conv_planes[3])
        self.conv5 = conv(conv_planes[3], conv_planes[4])
        self.conv6 = conv(conv_planes[4], conv_planes[5])
        self.conv7 = conv(conv_planes[5], conv_planes[6])
        self.pose_pred = nn.Conv2d(conv_planes[6], 6 * self.nb_ref_imgs, kernel_size=1, padding=0)
        if self.output_exp:
            upconv_planes = [256, 128, 64, 32, 16]
            self.upconv5 = upconv(conv_planes[4], upconv_planes[0])
            self.upconv4 = upconv(upconv_planes[0], upconv_planes[1])
            self.upconv3 = upconv(upconv_planes[1], upconv_planes[2])
            self.upconv2 = upconv(upconv_planes[2], upconv_planes[3])
            self.upconv1 = upconv(upconv_planes[3], upconv_planes[4])
            self.predict_mask4 = nn.Conv2d(upconv_planes[1], self.nb_ref_imgs, kernel_size=3, padding=1)
            self.predict_mask3 = nn.Conv2d(upconv_planes[2], self.nb_ref_imgs, kernel_size=3, padding=1)
            self.predict_mask2 = nn.Conv2d(upconv_planes[3], self.nb_ref_imgs, kernel_size=3, padding=1)
            self.predict_mask1 = nn.Conv2d(upconv_planes[4], self.nb_ref_imgs, kernel_size=3, padding=1)
        self._plan, self._plan_key = None, None

    def init_weights(self):                                         # posenet.py:57-62
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
                xavier_uniform_(m.weight.data)
                if m.bias is not None:
                    zeros_(m.bias)
        self._plan = None

    # ------------------------------------------------------------ packed weights
    def _prepare(self, dt):
        key = (dt,) + tuple((p.data_ptr(), p._version) for p in self.parameters())
        if self._plan is not None and self._plan_key == key:
            return self._plan
        P = {"conv1": K.PackedConv(self.conv1[0].weight, self.conv1[0].bias, dt, cin_pad=16)}
        for i in range(2, 8):
            c = getattr(self, f"conv{i}")[0]
            P[f"conv{i}"] = K.PackedConv(c.weight, c.bias, dt)
        P["pose_pred"] = K.PackedConv(self.pose_pred.weight, self.pose_pred.bias, dt)
        if self.output_exp:
            for i in range(1, 6):
                c = getattr(self, f"upconv{i}")[0]
                P[f"upconv{i}"] = K.PackedConv(c.weight, c.bias, dt, convt4=True)
            for i in range(1, 5):
                c = getattr(self, f"predict_mask{i}")
                P[f"predict_mask{i}"] = K.PackedConv(c.weight, c.bias, dt)
        self._plan, self._plan_key = P, key
        return P

    @staticmethod
    def _crop(x, h, w):
        """[:, :, 0:h, 0:w] of an NHWC activation (posenet.py:78-82)."""
        if x.shape[1] == h and x.shape[2] == w:
            return x
        return x[:, :h, :w].contiguous()

    @torch.no_grad()
    def forward(self, target_image, ref_imgs):
        assert len(ref_imgs) == self.nb_ref_imgs
        dt = next(self.parameters()).dtype
        if dt not in (torch.float32, torch.bfloat16):
            raise TypeError(f"PoseExpNet HIP path runs in float32 or bfloat16, not {dt}")
        P = self._prepare(dt)
        srcs = [target_image] + list(ref_imgs)
        if len(srcs) > 3:
            srcs = [srcs[0], torch.cat(srcs[1:], 1)]                # the gather takes <= 3 sources
        B, _, H, W = target_image.shape
        x = K.nchw_to_nhwc(srcs, 16, dt)                            # [B, H, W, 16] (9 real channels)
        feats, h, w = [], H, W
        for i in range(1, 8):
            x = K.conv2d(P[f"conv{i}"], x, B, h, w, stride=2, act=K.ACT_RELU)
            h, w = x.shape[1], x.shape[2]
            feats.append(x)
        pose = K.conv2d(P["pose_pred"], x, B, h, w, out_dtype=torch.float32)      # [B, h7, w7, 6 nref]
        pose = 0.01 * pose.mean(dim=(1, 2)).view(B, self.nb_ref_imgs, 6)
        if not self.output_exp:
            return ([None] * 4 if self.training else None), pose
        c1, c2, c3, c4, c5 = feats[:5]
        ups, u = [], c5
        for i, ref in ((5, c4), (4, c3), (3, c2), (2, c1), (1, None)):
            hh, ww = u.shape[1], u.shape[2]
            u = K.conv2d(P[f"upconv{i}"], u, B, hh, ww, out_layout=K.OUT_SHUFFLE2, act=K.ACT_RELU)
            u = self._crop(u, *((ref.shape[1], ref.shape[2]) if ref is not None else (H, W)))
            ups.append(u)
        u4, u3, u2, u1 = ups[1], ups[2], ups[3], ups[4]
        masks = []
        for i, uu in ((1, u1), (2, u2), (3, u3), (4, u4)):
            masks.append(K.conv2d(P[f"predict_mask{i}"], uu, B, uu.shape[1], uu.shape[2], out_layout=K.OUT_NCHW,
                                  act=K.ACT_SIGMOID, out_dtype=torch.float32))
        if self.training:
            return masks, pose
        return masks[0], pose
