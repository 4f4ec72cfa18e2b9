// Poisoned stand-in for the reference header normEncoderMDP.h (test fixture): a drop-in build must find
// include/norm_fec/ first; reaching this file means the reference header would be used.
#error "reference header normEncoderMDP.h was picked up instead of include/norm_fec"
