"""Drop-in for python/src/custom_models/models.py: TICA_LapDropout (the paper's PriGumbel model,
models.py:28-82) with its (eeg_txt_input, eeg_txt_mask, act_img_input, act_img_mask, epsilon,
hard) forward signature."""
from eegfusion.modules import TICA_LapDropout  # noqa: F401
