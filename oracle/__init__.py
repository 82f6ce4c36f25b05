"""CPU oracle of the ORB front-end -- TEST INFRASTRUCTURE ONLY (see orbref.h)."""
