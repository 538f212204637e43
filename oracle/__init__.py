"""CPU restatement of the reference path — TEST INFRASTRUCTURE ONLY (see oracle.h)."""
