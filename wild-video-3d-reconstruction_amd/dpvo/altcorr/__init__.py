from .correlation import corr, corr_pyramid, corr_pyramid_mfma, corr_pyramid_staged, patchify
