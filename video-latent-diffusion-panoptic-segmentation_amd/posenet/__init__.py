"""posenet — drop-in for the reference's posenet/ package (PoseExpNet, BASELINE config 5)."""
