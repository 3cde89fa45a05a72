"""Reaction-diffusion model family (reference models/reaction/)."""
