"""Simulation model: data containers, genetics, kinetics, world and genome factories."""
