"""CPU restatement of the reference's denoising path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import anything from this package, and only as the *checker* (or as the timed
CPU baseline).  The product package (``video-latent-diffusion-panoptic-segmentation_amd``)
never imports it: its ops run through the HIP C-ABI library and fail loudly when that
library is missing.

Modules and how each is pinned:

* ``codec``  bit-channel mask codec (numpy, integer/byte exact)
             pinned: tests/golden/codec.npz (reference functions + the reference's own
             sample_outputs/ known-answer PNGs)
* ``ddim``   DDIM noise schedule / step / add_noise / remove_noise (torch fp32, CPU)
             pinned: tests/golden/ddim.npz
* ``vae``    GeneralVAESeg encode / decode conv stacks (torch fp32, CPU)
             pinned: tests/golden/vae.npz
* ``unet``   SD-1.x UNet2DConditionModel graph as configured by the reference (torch fp32, CPU)
             **parity unpinned** w.r.t. the reference: its arithmetic lives in the
             un-vendored ``diffusers`` package.  It follows the public
             diffusers structure and is pinned per op against
             torch.nn.functional only.
* ``dvpq``   eval/eval_dvpq.py ``vpq_eval`` restatement (numpy)
             pinned: tests/golden/vpq.npz
"""
