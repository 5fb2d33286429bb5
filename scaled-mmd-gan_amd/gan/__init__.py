"""MI355X-native Scaled-MMD-GAN training path (drop-in for the reference's gan/ tree)."""
